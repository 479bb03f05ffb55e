"""CPU model of path 4's device chain (k_stream_chain, sm_decompress.hip) on a stream: how many
path elements the chain takes from the index's entry records, from the deep records, or by its own
serial walk (dev_walk, the slow case).  Design tool:  python3 tools/chain_model.py STREAM... [--levels K]
Streams from tools/dump_streams.py (gpurun_out/streams/).  --runs: the round-5 chain's parallel
runs (how many elements the workgroup writes, how many steps stay serial)."""
import argparse

KC = 1024        # kSmallChunk
NEXTONLY = False  # extra chains only for exits inside the next chunk
ENTRIES = 64     # kIdxEntries


def varint(b):
    v, s, i = 0, 0, 0
    while True:
        x = b[i]
        v |= (x & 0x7F) << s
        i += 1
        if x < 0x80:
            return v, i
        s += 7


def tag(b, p):
    """(size in the stream, output bytes) of the tag at p, bytes past the end read as zero."""
    def at(i):
        return b[i] if i < len(b) else 0
    c = at(p)
    t = c & 3
    if t == 0:
        n = c >> 2
        if n < 60:
            return 1 + n + 1, n + 1
        tl = n - 59
        tr = 0
        for j in range(tl):
            tr |= at(p + 1 + j) << (8 * j)
        return 1 + tl + tr + 1, tr + 1
    if t == 1:
        return 2, ((c >> 2) & 7) + 4
    if t == 2:
        return 3, (c >> 2) + 1
    return 5, (c >> 2) + 1


def walk(b, p, lim):
    o = 0
    while p < lim:
        s, ob = tag(b, p)
        p += s
        o += ob
    return p, o


def model(b, levels, distinct=1):
    """distinct: deep records for up to that many distinct exits of the chunk's 64 entry lanes
    (1: lane 0's exit only, the kernel as built)."""
    N = len(b)
    size, ip0 = varint(b)
    nch = (N - ip0 + KC - 1) // KC
    deep = []   # per chunk: a list of record chains, each a list of (x, exit) levels
    for c in range(nch):
        s = ip0 + c * KC
        exits = []
        for l in range(ENTRIES if distinct > 1 else 1):
            x, _ = walk(b, s + l, min(s + KC, N - 1))
            if l and NEXTONLY and not (x < s + 2 * KC):
                continue  # (an entry lane's exit past the next chunk: not used)
            if x not in exits:
                exits.append(x)
        chains = []
        for x in exits[:distinct]:
            lv = []
            for _ in range(levels):
                dl = (x - ip0) // KC
                db = ip0 + dl * KC
                if not (x < N - 1 and x - db >= ENTRIES):
                    break
                dex, _ = walk(b, x, min(db + KC, N - 1))
                lv.append((x, dex))
                x = dex
            chains.append(lv)
        deep.append(chains)
    y, n_rec, n_deep, n_walk = ip0, 0, 0, 0
    cprev, dsrc, dlev = None, None, 0
    walk_bytes = 0
    while y < N - 1:
        c = (y - ip0) // KC
        base = ip0 + c * KC
        l = y - base
        if l < ENTRIES:
            ex, _ = walk(b, y, min(base + KC, N - 1))
            n_rec += 1
            dsrc = None
        else:
            hit = None
            if dsrc is not None and dlev + 1 < len(deep[dsrc[0]][dsrc[1]]) and deep[dsrc[0]][dsrc[1]][dlev + 1][0] == y:
                hit = (dsrc, dlev + 1)
            elif cprev is not None:
                for i, ch in enumerate(deep[cprev]):
                    if ch and ch[0][0] == y:
                        hit = ((cprev, i), 0)
                        break
            ex, _ = walk(b, y, min(base + KC, N - 1))
            if hit:
                n_deep += 1
                dsrc, dlev = hit
            else:
                n_walk += 1
                walk_bytes += min(base + KC, N - 1) - y
                dsrc = None
        cprev = c
        y = ex
    return nch, n_rec, n_deep, n_walk, walk_bytes


def model_runs(b, levels, distinct, deeplink=True, min_run=8):
    """The round-5 chain (k_stream_chain): chunk links (E(c) into a recorded entry that exits at
    E(c'), through chain 0's deep records when deeplink), pointer-jumped; wave 0 steps serially
    and hands a run to the workgroup at an entry record with >= min_run links ahead.  Returns
    (runs, run elements, serial record steps, serial deep steps, walks)."""
    N = len(b)
    size, ip0 = varint(b)
    nch = (N - ip0 + KC - 1) // KC
    lim = lambda c: min(ip0 + c * KC + KC, N - 1)
    E = [walk(b, ip0 + c * KC, lim(c))[0] for c in range(nch)]
    chain0 = []  # chain 0's deep levels per chunk: list of (x, exit)
    for c in range(nch):
        lv, x = [], E[c]
        for _ in range(levels):
            dl = (x - ip0) // KC
            if not (x < N - 1 and x - (ip0 + dl * KC) >= ENTRIES):
                break
            dex = walk(b, x, lim(dl))[0]
            lv.append((x, dex))
            x = dex
        chain0.append(lv)
    link, cnt = [None] * nch, [1] * nch
    for c in range(nch):
        X, k, nd = E[c], 0, 0
        while X < N - 1:
            cx, lx = (X - ip0) // KC, (X - ip0) % KC
            if cx >= nch or cx <= c:
                break
            if lx < ENTRIES:
                if walk(b, X, lim(cx))[0] == E[cx]:
                    link[c], cnt[c] = cx, 1 + nd
                break
            if not deeplink or k >= len(chain0[c]) or chain0[c][k][0] != X:
                break
            X, k, nd = chain0[c][k][1], k + 1, nd + 1
    D = [0] * nch
    for c in range(nch - 1, -1, -1):
        D[c] = 0 if link[c] is None else 1 + D[link[c]]
    # the serial chain (model() rules) with runs
    deep = []
    for c in range(nch):  # deep records as model() builds them (distinct chains, levels)
        s0 = ip0 + c * KC
        exits = []
        for l in range(ENTRIES if distinct > 1 else 1):
            x, _ = walk(b, s0 + l, lim(c))
            if l and NEXTONLY and not (x < s0 + 2 * KC):
                continue
            if x not in exits:
                exits.append(x)
        chains = []
        for x in exits[:distinct]:
            lv = []
            for _ in range(levels):
                dl = (x - ip0) // KC
                if not (x < N - 1 and x - (ip0 + dl * KC) >= ENTRIES):
                    break
                dex = walk(b, x, lim(dl))[0]
                lv.append((x, dex))
                x = dex
            chains.append(lv)
        deep.append(chains)
    y, cprev, dsrc, dlev = ip0, None, None, 0
    runs = run_el = s_rec = s_deep = s_walk = 0
    while y < N - 1:
        c = (y - ip0) // KC
        l = y - (ip0 + c * KC)
        ex, _ = walk(b, y, lim(c))
        if l < ENTRIES:
            if ex == E[c] and D[c] >= min_run:
                runs += 1
                r = c
                while link[r] is not None:
                    run_el += cnt[r]
                    r = link[r]
                run_el += 1
                y, cprev, dsrc = E[r], r, None
                continue
            s_rec += 1
            dsrc = None
        else:
            hit = None
            if dsrc is not None and dlev + 1 < len(deep[dsrc[0]][dsrc[1]]) and deep[dsrc[0]][dsrc[1]][dlev + 1][0] == y:
                hit = (dsrc, dlev + 1)
            elif cprev is not None:
                for i, ch in enumerate(deep[cprev]):
                    if ch and ch[0][0] == y:
                        hit = ((cprev, i), 0)
                        break
            if hit:
                s_deep += 1
                dsrc, dlev = hit
            else:
                s_walk += 1
                dsrc = None
        cprev = c
        y = ex
    return runs, run_el, s_rec, s_deep, s_walk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("streams", nargs="+")
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--distinct", type=int, default=1, help="deep-record chains per chunk (distinct entry exits)")
    ap.add_argument("--next-only", action="store_true", help="extra chains only for exits inside the next chunk")
    ap.add_argument("--chunk", type=int, default=1024, help="index chunk bytes (kSmallChunk / kSmallChunkFine)")
    ap.add_argument("--runs", action="store_true", help="the round-5 parallel-run chain (model_runs)")
    ap.add_argument("--no-deeplink", action="store_true", help="--runs: links through entry records only")
    a = ap.parse_args()
    global NEXTONLY, KC
    NEXTONLY = a.next_only
    KC = a.chunk
    if a.runs:
        print("%-40s %6s %8s %8s %8s %8s" % ("stream", "runs", "run el", "ser rec", "ser deep", "walks"))
        for f in a.streams:
            b = open(f, "rb").read()
            print("%-40s %6d %8d %8d %8d %8d" % ((f.split("/")[-1],) + model_runs(b, a.levels, a.distinct, not a.no_deeplink)))
        return
    print("%-40s %6s %6s %6s %6s %8s" % ("stream", "chunks", "rec", "deep", "walks", "walk B"))
    for f in a.streams:
        b = open(f, "rb").read()
        print("%-40s %6d %6d %6d %6d %8d" % ((f.split("/")[-1],) + model(b, a.levels, a.distinct)))


if __name__ == "__main__":
    main()
