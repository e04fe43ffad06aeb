#!/usr/bin/env python3
"""CPU model of the single-pass decoder's dependency rounds (research tool).

Parses oracle-compressed 4 MiB blocks into sequences, cuts them into the
kernel's 1 KiB chunk tables, and counts per table: matches pending after round 1
under the kernel's rule (source before the table, or remappable through <= 8
single-piece hops: remap_src), and what a segment-wise chase would need instead
(every pending match split at the piece boundaries of its source, each segment
chased through matches to literal bytes or pre-table output)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import oracle as O


def parse(comp):
    seqs, p, n, y = [], 0, len(comp), 0
    while p < n:
        t = comp[p]; p0 = p; p += 1
        ll = t >> 4
        if ll == 15:
            while True:
                b = comp[p]; p += 1; ll += b
                if b != 255: break
        lit = p; p += ll
        if p >= n:
            seqs.append((p0, y, ll, lit, 0, 0)); y += ll; break
        off = comp[p] | (comp[p + 1] << 8); p += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = comp[p]; p += 1; ml += b
                if b != 255: break
        ml += 4
        seqs.append((p0, y, ll, lit, off, ml)); y += ll + ml
    return seqs


def tables(seqs):
    out, i, ip = [], 0, 0
    while i < len(seqs):
        j = i
        while j < len(seqs) and seqs[j][0] < ip + 1024:
            j += 1
        if j == i: j = i + 1
        out.append(seqs[i:j]); ip = seqs[j - 1][0] + 1 if j < len(seqs) else 1 << 62
        ip = max(ip, seqs[i][0] + 1024) if j - i > 1 else seqs[j - 1][0] + 1
        if j < len(seqs): ip = seqs[j][0]
        i = j
    return out


def model(comp):
    seqs = parse(comp)
    st = dict(tables=0, matches=0, pend=0, pend_per=0, segs=0, hops=0, maxhops=0, rounds=0, gsegs=0, grp_g=0, grp_s=0,
              fail8=0)
    for T in tables(seqs):
        st["tables"] += 1
        O_ = T[0][1]
        starts = [s[1] for s in T]
        import bisect

        def piece(pos):   # (kind, seq index, piece end): kind 0 literal, 1 match
            k = bisect.bisect_right(starts, pos) - 1
            _, y, ll, lit, off, ml = T[k]
            return (0, k, y + ll) if pos < y + ll else (1, k, y + ll + ml)

        pend = []
        for k, (_, y, ll, lit, off, ml) in enumerate(T):
            if ml == 0: continue
            st["matches"] += 1
            ms = y + ll; rs = ms - off; re = rs + ml; per = off < ml
            if (ms if per else re) <= O_: continue
            ok = False
            if not per:
                a, b = rs, re
                for _ in range(8):
                    if b <= O_: ok = True; break
                    if a < O_: break
                    kind, kk, pe = piece(a)
                    if b > pe: break
                    if kind == 0: ok = True; break
                    a -= T[kk][4]; b -= T[kk][4]
            if not ok:
                pend.append(k); st["pend"] += 1; st["pend_per"] += per
        # segment chase for the pending ones
        lane_g = {}; lane_s = {}
        for k in pend:
            _, y, ll, lit, off, ml = T[k]
            if off < ml: continue
            pos, end = y + ll, y + ll + ml
            failed = False
            while pos < end:
                a = pos - off; n = min(end - pos, 16); h = 0
                while a >= O_:
                    kind, kk, pe = piece(a)
                    n = min(n, pe - a)
                    if kind == 0: break
                    a -= T[kk][4]; h += 1
                if a < O_:
                    n = min(n, O_ - a); st["gsegs"] += 1
                    lane_g[k] = lane_g.get(k, 0) + 1
                lane_s[k] = lane_s.get(k, 0) + 1
                if h > 8: failed = True
                st["segs"] += 1; st["hops"] += h; st["maxhops"] = max(st["maxhops"], h)
                pos += n
            st["fail8"] += failed
        for g in range(0, len(T), 64):
            st["grp_g"] += max([lane_g.get(k, 0) for k in range(g, g + 64)] + [0])
            st["grp_s"] += max([lane_s.get(k, 0) for k in range(g, g + 64)] + [0])
        # rounds under the current rule (pending match ready when its source meets no pending match)
        done = set(range(len(T))) - set(pend)
        r = 0
        rem = list(pend)
        while rem:
            r += 1
            nxt = []
            for k in rem:
                _, y, ll, lit, off, ml = T[k]
                ms = y + ll; rs = ms - off; re = ms if off < ml else rs + ml
                blocked = any(not (T[j][1] + T[j][2] + T[j][5] <= rs or T[j][1] + T[j][2] >= re)
                              for j in rem if j != k and j not in nxt and T[j][1] + T[j][2] < re)
                (nxt if blocked else []).append(k) if blocked else None
            if len(nxt) == len(rem): break
            rem = nxt
        st["rounds"] += r
    return st


if __name__ == "__main__":
    for gen in sys.argv[1].split(","):
        src = O.generate(gen, 1, 4 << 20)
        comp = O.compress_block_bytes(src).tobytes()
        s = model(comp)
        t = s["tables"]
        print(gen, "ratio %.2f" % (len(src) / len(comp)), "tables", t,
              "matches/table %.1f" % (s["matches"] / t), "pending/table %.2f (periodic %.2f)" % (s["pend"] / t, s["pend_per"] / t),
              "segments/pending %.2f" % (s["segs"] / max(1, s["pend"])), "hops/segment %.2f max %d" % (s["hops"] / max(1, s["segs"]), s["maxhops"]),
              "rounds/table %.2f" % (s["rounds"] / t),
              "global segs/pending %.2f" % (s["gsegs"] / max(1, s["pend"])),
              "per table: sum over groups of max-lane segs %.2f, global segs %.2f; >8 hops %.2f" % (s["grp_s"] / t, s["grp_g"] / t, s["fail8"] / t), flush=True)
