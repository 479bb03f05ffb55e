"""Shared fixtures.  `gpu`-marked tests need an MI355X (run via gpurun); everything else runs
on CPU.  The oracle (oracle/) is test infrastructure: imported here only as the checker."""
import ctypes
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# test/runtests.jl:8-24
ROUNDTRIP_FILES = [
    "alice29.txt", "asyoulik.txt", "html", "html_x_4", "kppkn.gtb", "lcet10.txt", "fireworks.jpeg",
    "geo.protodata", "paper-100k.pdf", "plrabn12.txt", "urls.10K", "random1.bin", "random2.bin",
    "random3.bin", "smallrandom1.bin",
]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run through gpurun)")


def load_package():
    """Import snappy.jl_amd/ (the directory name is not a valid identifier)."""
    if "snappy_jl_amd" in sys.modules:
        return sys.modules["snappy_jl_amd"]
    pkg_dir = os.path.join(ROOT, "snappy.jl_amd")
    spec = importlib.util.spec_from_file_location("snappy_jl_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["snappy_jl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def read_testfile(name):
    with open(os.path.join(TESTDATA, name), "rb") as fh:
        return fh.read()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def sm():
    return load_package()


@pytest.fixture(scope="session")
def libsnappy():
    """libsnappy 1.1.8 from the image (an independent decoder/encoder); skip if absent."""
    path = "/opt/conda/lib/libsnappy.so.1"
    if not os.path.exists(path):
        pytest.skip("libsnappy not present")
    L = ctypes.CDLL(path)

    class Lib:
        @staticmethod
        def compress(x):
            out = ctypes.create_string_buffer(32 + len(x) + len(x) // 6 + 8)
            ol = ctypes.c_size_t(len(out))
            assert L.snappy_compress(x, ctypes.c_size_t(len(x)), out, ctypes.byref(ol)) == 0
            return out.raw[: ol.value]

        @staticmethod
        def uncompress(x):
            n = ctypes.c_size_t(0)
            if L.snappy_uncompressed_length(x, ctypes.c_size_t(len(x)), ctypes.byref(n)) != 0:
                return None
            out = ctypes.create_string_buffer(max(n.value, 1))
            if L.snappy_uncompress(x, ctypes.c_size_t(len(x)), out, ctypes.byref(n)) != 0:
                return None
            return out.raw[: n.value]

    return Lib


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
