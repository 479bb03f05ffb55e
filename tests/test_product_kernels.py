"""The shipped library carries product kernels only.

Reads the gfx950 code objects embedded in snappy.jl_amd/libsnappy_mi355x.so (the .hip_fatbin
section: one clang offload bundle per translation unit) with a minimal ELF reader, lists their
kernel descriptors (`<name>.kd` symbols) and device variables, and checks them against the
product's kernel list.  A diagnostic kernel (the round-4 queue decoder, a probe) or a stamp buffer
compiled into the product fails the test.  CPU only: nothing is launched."""
import os
import re
import struct

from conftest import ROOT

LIB = os.path.join(ROOT, "snappy.jl_amd", "libsnappy_mi355x.so")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# every kernel the product launches (sm_api.hip launch_* paths), by unmangled base name
PRODUCT_KERNELS = {
    "k_compress_exact", "k_literal_screen", "k_compress_sc", "k_compress_sc_span",
    "k_gather", "k_gather16", "k_gather_parts", "k_frag_plan", "k_place",
    "k_decompress", "k_decompress_one", "k_decompress_frags", "k_validate", "k_uncompressed_length",
    "k_stream_index", "k_stream_chain", "k_origin_fill", "k_origin_fill_dev", "k_origin_resolve",
    "k_origin_gather", "k_small_resolve", "k_to_host", "k_path_check", "k_literal_spans",
}
DIAGNOSTIC = re.compile(r"_q$|queue|stamp|probe|abl|dup|debug", re.I)


def _elf_sections(data):
    """(name, offset, size, type, link, entsize) of an ELF64 little-endian file's sections."""
    assert data[:4] == b"\x7fELF" and data[4] == 2 and data[5] == 1
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    raw = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    strtab = raw[shstrndx]
    out = []
    for (name, typ, _flags, _addr, off, size, link, _info, _align, entsize) in raw:
        s = data[strtab[4] + name: data.index(b"\0", strtab[4] + name)].decode()
        out.append((s, off, size, typ, link, entsize))
    return out


def _symbols(data):
    secs = _elf_sections(data)
    names = []
    for (name, off, size, typ, link, entsize) in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][1]
        for k in range(size // entsize):
            st_name, = struct.unpack_from("<I", data, off + k * entsize)
            if st_name:
                names.append(data[stroff + st_name: data.index(b"\0", stroff + st_name)].decode())
    return names


def _code_objects(lib_bytes):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin."""
    fat = [s for s in _elf_sections(lib_bytes) if s[0] == ".hip_fatbin"]
    assert fat, "no .hip_fatbin section: not a HIP library"
    _, off, size, _, _, _ = fat[0]
    blob = lib_bytes[off: off + size]
    cos, pos = [], 0
    while True:
        i = blob.find(BUNDLE_MAGIC, pos)
        if i < 0:
            break
        n, = struct.unpack_from("<Q", blob, i + 24)
        p = i + 32
        for _ in range(n):
            eoff, esize, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p: p + tl].decode()
            p += tl
            if "gfx950" in triple:
                cos.append(blob[i + eoff: i + eoff + esize])
        pos = i + 1
    return cos


def _base_name(mangled):
    """k_... from an Itanium-mangled sm:: kernel name (_ZN2sm<len><name>...)."""
    m = re.match(r"_ZN2sm(\d+)", mangled)
    if not m:
        return mangled
    n = int(m.group(1))
    return mangled[m.end(): m.end() + n]


def product_kernels():
    data = open(LIB, "rb").read()
    kernels, variables = set(), set()
    for co in _code_objects(data):
        for s in _symbols(co):
            if s.endswith(".kd"):
                kernels.add(_base_name(s[:-3]))
            elif s.startswith("_ZN2sm") and not s.endswith(".kd"):
                variables.add(s)
    return kernels, variables


def test_code_objects_are_gfx950():
    cos = _code_objects(open(LIB, "rb").read())
    assert len(cos) >= 4  # one per translation unit with kernels
    for co in cos:
        # e_machine EM_AMDGPU (224)
        assert struct.unpack_from("<H", co, 0x12)[0] == 224


def test_shipped_kernels_are_product_kernels():
    kernels, variables = product_kernels()
    assert "k_compress_sc" in kernels and "k_decompress" in kernels and "k_place" in kernels
    unknown = kernels - PRODUCT_KERNELS
    assert not unknown, "kernels outside the product list in the shipped library: %s" % sorted(unknown)
    diag = sorted(k for k in kernels if DIAGNOSTIC.search(k))
    assert not diag, "diagnostic kernels in the shipped library: %s" % diag
    # no device-side diagnostic buffers either (stamp arrays, a queue counter)
    dvars = sorted(v for v in variables if DIAGNOSTIC.search(v))
    assert not dvars, "diagnostic device variables in the shipped library: %s" % dvars


def test_product_sources_have_no_diagnostic_switches():
    """The product translation units carry no ablation / duplication / stamp / queue switches:
    a mis-set flag cannot ship a variant (round-6 cleanup; the kernels' disassembly was
    unchanged by it)."""
    csrc = os.path.join(ROOT, "snappy.jl_amd", "csrc")
    pat = re.compile(r"\b(SC_ABL|SC_DUP|SC_GC|SC_SPAN_ABL|SM_STAMP|SM_ABLATE_D|SM_DUP_D|SM_DEC_QUEUE|"
                     r"SM_IDX_NOLANES|STAMP_FLUSH|k_decompress_q)\b")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")):
            hits = [i + 1 for i, line in enumerate(open(os.path.join(csrc, f))) if pat.search(line)]
            assert not hits, "%s: diagnostic switches at lines %s" % (f, hits)
