"""Turn the PMC passes of tools/pmc_run.sh into profiles/<round>_pmc.json (bench.py's `traffic`).

Usage: python tools/pmc_json.py <round-dir> <out.json>
  <round-dir>/pmc_compress and <round-dir>/pmc_uncompress hold the rocprofv3 --pmc passes.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read, so it is doubled.  Calibration on our own access pattern: the
fast compressor reads every input byte exactly once with 16 B/lane loads, and 2 x FETCH_SIZE
matches the algorithmic input bytes to within 1% (profiles/r01_pmc.json, "calibration").
The decoder's copy-source re-reads are 8 B/lane and stay uncalibrated (noted per kernel).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402

# bench.py roofline key -> (pass directory, rocprof kernel names summed per launch).  A fast-mode
# compress call is two kernels: the incompressible screen and the parse (which returns at once
# for the blocks the screen emitted).
KERNELS = {"compress_fast": ("pmc_compress", ["k_literal_screen", "k_compress_sc<0>"]),
           "uncompress": ("pmc_uncompress", ["k_decompress("]),
           "compress_fast_random": ("pmc_compress_random", ["k_literal_screen", "k_compress_sc<0>"]),
           "uncompress_random": ("pmc_uncompress_random", ["k_decompress("]),
           "compress_fragments": ("pmc_compress_fragments", ["k_literal_screen", "k_compress_sc<0>"]),
           "uncompress_reference_streams": ("pmc_uncompress_reference", ["k_decompress("])}
IN_BYTES = 10000 * 65536  # uncompressed bytes per launch (tools/pmc_run.sh BLOCKS=10000)
IN_BYTES_FRAG = 675282944  # config 5's stream (bench.CONFIG5_BYTES)


def main(root, out_path, library=None, commit=None):
    res = {"source": "rocprofv3 --kernel-trace --pmc, one pass per counter group (tools/pmc_run.sh)",
           "units": "bytes per launch (10000 x 64 KiB blocks: text, or uniform random for *_random; "
                    "compress_fragments: config 5's 10,304 fragments)",
           # the build the passes measured (sm_version() in the kbench logs) and the commit they ran at:
           # bench.py labels `traffic` with them and flags a file from another build
           "library": library, "commit": commit}
    for key, (sub, knames) in KERNELS.items():
        per = {}
        for kn in knames:
            d = summarise(os.path.join(root, sub), kn)
            if d:
                per[next(iter(d.keys()))] = next(iter(d.values()))
        if not per:
            continue
        fetch = sum(c.get("FETCH_SIZE", 0.0) for c in per.values()) * 1024.0
        write = sum(c.get("WRITE_SIZE", 0.0) for c in per.values()) * 1024.0
        res[key] = {
            "kernels": [k[:60] for k in per],
            "fetch_size_bytes_raw": fetch,
            "write_size_bytes": write,
            "hbm_bytes_per_launch": 2.0 * fetch + write,
            "counters": {k[:60]: {n: v for n, v in sorted(c.items())} for k, c in per.items()},
            # issue-side figures per uncompressed input byte (10,000 x 64 KiB per launch)
            "per_input_byte": {n: sum(c.get(n, 0.0) for c in per.values()) / (IN_BYTES_FRAG if "fragments" in key else IN_BYTES)
                               for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH")},
        }
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in res.items() if isinstance(v, dict)}))


def library_of(root):
    """The library version the PMC passes' kbench runs printed (tools/kbench.py: 'library ...')."""
    for sub in ("pmc_compress", "pmc_uncompress"):
        d = os.path.join(root, sub)
        for f in sorted(os.listdir(d)) if os.path.isdir(d) else []:
            if f.endswith(".log"):
                for line in open(os.path.join(d, f)):
                    if line.startswith("library "):
                        return line.split(None, 1)[1].strip()
    return None


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], library_of(sys.argv[1]), sys.argv[3] if len(sys.argv) > 3 else None)
