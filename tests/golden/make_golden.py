"""Generate tests/golden/golden.json (committed fixture) from the CPU oracle.

The reference (Julia) cannot run in this container, so the golden vectors
are the oracle's reference-mode output.  They are cross-checked against the independent
transliteration table of SURVEY.md 8(c) (`SURVEY_TABLE` below, copied from the survey's
probe) and, in compat mode, against libsnappy 1.1.8 -- tests/test_oracle.py re-asserts both.

Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

# file -> (N, C reference mode, sha256 of reference-mode bytes)
SURVEY_TABLE = {
    "alice29.txt": (152089, 88039, "b3707b512e4cf11c6bde9603be53dfef10f147eb5c7c547ffbeb93ed3aeeaf66"),
    "asyoulik.txt": (125179, 77503, "4bf8701f8c369f13e679f52e938c8630d2a2920eba4003bfeeced8522d984aa9"),
    "html": (102400, 22843, "c7c94425c2b3516cf3d1c9824391b8453beb544f38dfdfa90eb8126103234b5a"),
    "html_x_4": (409600, 92234, "11e53110e963fa6dd4ef3d726cf2d897a7ab689c8edb90ccab3f462ef21872f3"),
    "kppkn.gtb": (184320, 69526, "b6513d28c84b3715f02a2697ddb3f6b56aab8f09f0b5950075762912ae5ae8d9"),
    "lcet10.txt": (426754, 234662, "39bd4948c8743f4862e7a83fc36113f1db80712a0feb7545c048d43d26354268"),
    "fireworks.jpeg": (123093, 123034, "4da5e82d77ebe3d77e4f827a294562df17b5dcf37dcdb30d516ee8544d3164a6"),
    "geo.protodata": (118588, 23335, "84356d0f45f9cf8547834eabaa8d4ec569c3e71c505828ab3321ffbd35370d11"),
    "paper-100k.pdf": (102400, 85304, "ad668e5050689de4486cca4851a67b81731ff77ae920dc78da2e5fc9ca36d7e5"),
    "plrabn12.txt": (481861, 319267, "30915f0a26ae2b882e7d8a6951dc3e844c8dd615b0a1a21c6dd69e8c8f958337"),
    "urls.10K": (702087, 335506, "a0b5838bba64270a4fd4ca45eae8fe79469fd3ac1e3eab7208b5cbce9fd6d810"),
    "random1.bin": (463999, 127284, "022e2e41ae533e03b120d0f29178bc16ccd0fdac9ff987a63fee771935355941"),
    "random2.bin": (335830, 92416, "cd9d24141fa3f2273b60ac3cb636defa56f7f9d523302985890d4aa8daebbeab"),
    "random3.bin": (408750, 108560, "fb1d85c2dcbdba67c02b47c73333e0be99005082b5b39ef54bd064c524d326f8"),
    "smallrandom1.bin": (427, 419, "d2b59e74172aa7fb67961f5d25fa16be95c7134f239e3650b88424f806ec0e51"),
    "sample-tweet.json": (12836, 3469, "3dd7721222ebdd07cc772ec3cf2e73da9b7523ef85884f737c0ded0b3496107d"),
}

# test/runtests.jl:127-137 edge strings
EDGE_STRINGS = [
    b"", b"a", b"ab", b"abc",
    b"aaaaaaa" + b"b" * 16 + b"aaaaa" + b"abc",
    b"aaaaaaa" + b"b" * 256 + b"aaaaa" + b"abc",
    b"aaaaaaa" + b"b" * 2047 + b"aaaaa" + b"abc",
    b"aaaaaaa" + b"b" * 65536 + b"aaaaa" + b"abc",
    b"abcaaaaaaa" + b"b" * 65536 + b"aaaaa" + b"abc",
]


REFERENCE_INTERNAL = "/root/reference/src/internal.jl"


def char_table_from_reference():
    """CHAR_TABLE values (src/internal.jl:47-80) as data, for the derived-table check."""
    import re
    src = open(REFERENCE_INTERNAL).read()
    body = src[src.index("CHAR_TABLE = UInt16["):]
    body = body[: body.index("]")]
    vals = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]{4}", body)]
    assert len(vals) == 256
    return vals


def main():
    out = {"corpus": {}, "edge_strings": []}
    if os.path.exists(REFERENCE_INTERNAL):
        out["char_table"] = char_table_from_reference()
    else:
        out["char_table"] = json.load(open(os.path.join(HERE, "golden.json")))["char_table"]
    for f in sorted(SURVEY_TABLE):
        raw = open(os.path.join(HERE, "testdata", f), "rb").read()
        ref = O.compress(raw)
        com = O.compress(raw, compat=True)
        assert O.uncompress(ref) == raw
        n, c, sha = SURVEY_TABLE[f]
        assert (len(raw), len(ref), hashlib.sha256(ref).hexdigest()) == (n, c, sha), f
        out["corpus"][f] = {
            "n": len(raw),
            "c_reference": len(ref),
            "sha256_reference": hashlib.sha256(ref).hexdigest(),
            "c_compat": len(com),
            "sha256_compat": hashlib.sha256(com).hexdigest(),
        }
    for s in EDGE_STRINGS:
        ref = O.compress(s)
        rec = {"input_sha256": hashlib.sha256(s).hexdigest(), "n": len(s),
               "c_reference": len(ref), "sha256_reference": hashlib.sha256(ref).hexdigest()}
        if len(ref) <= 64:
            rec["hex_reference"] = ref.hex()
        out["edge_strings"].append(rec)
    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote golden.json")


if __name__ == "__main__":
    main()
