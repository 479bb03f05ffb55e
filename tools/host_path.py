"""PCIe-inclusive single-buffer path (design tool, GPU box): sm_compress / sm_uncompress from host
buffers on config 5 (one 644 MiB stream), best of 5, with the bench's check.  SNAPPY_MI355X_LIB
selects a diagnostic build."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    sm = bench.load_package()
    big = bench.large_corpus()
    for _ in range(2):
        print(bench.config5_host_stream(sm, big, reps=5), flush=True)


if __name__ == "__main__":
    main()
