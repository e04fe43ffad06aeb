# CPU model (round 6): how much of a block's output run-level ("piece") pointers could resolve
# before the small path's byte-level pointer jumping. A match whose first period lies inside one earlier
# piece (a literal run, or the first period of a match) points at that piece with a delta; pieces are
# resolved by doubling over those pointers; the rest would keep byte pointers.
#   python tools/proto/piece_pointer_model.py tiles216,copy,text,runs
import sys, numpy as np, bisect
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__file__), '..', '..'))
from oracle import oracle as O

def parse(c):
    c = bytes(c); i = 0; x = 0; seqs = []   # (xs, lit_src, ll, off, ml)
    n = len(c)
    while i < n:
        t = c[i]; i += 1
        ll = t >> 4
        if ll == 15:
            while True:
                b = c[i]; i += 1; ll += b
                if b != 255: break
        src = i; i += ll
        if i >= n:
            seqs.append((x, src, ll, 0, 0)); x += ll; break
        off = c[i] | (c[i+1] << 8); i += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = c[i]; i += 1; ml += b
                if b != 255: break
        ml += 4
        seqs.append((x, src, ll, off, ml)); x += ll + ml
    return seqs

def model(kind, seed, rounds=12):
    src = O.generate(kind, seed, 4 << 20)
    c = O.compress_block_bytes(src)
    S = parse(c)
    N = len(S)
    starts = [s[0] for s in S]
    # state: ('L', p) / ('H', y) / ('P', q, d) / ('B',)
    st = [None] * N
    for k, (xs, ls, ll, off, ml) in enumerate(S):
        if ml == 0: st[k] = ('N',); continue
        ms = xs + ll; y0 = ms - off; span = min(ml, off)
        if y0 < 0:
            st[k] = ('H', y0) if y0 + span <= 0 else ('B',); continue
        q = bisect.bisect_right(starts, y0) - 1
        qx, qs, qll, qoff, qml = S[q]
        if y0 < qx + qll:
            st[k] = ('L', qs + y0 - qx) if y0 + span <= qx + qll else ('B',)
        else:
            qms = qx + qll; d = y0 - qms
            if y0 + span > qms + qml: st[k] = ('B',); continue
            per = min(qml, qoff)
            if d + span > per:
                if d // per == (d + span - 1) // per: d %= per
                else: st[k] = ('B',); continue
            st[k] = ('P', q, d)
    r_used = 0
    for r in range(rounds):
        ch = False
        new = list(st)
        for k in range(N):
            s = st[k]
            if s[0] != 'P': continue
            t = st[s[1]]
            ch = True
            if t[0] == 'L': new[k] = ('L', t[1] + s[2])
            elif t[0] == 'H': new[k] = ('H', t[1] + s[2])
            elif t[0] == 'P': new[k] = ('P', t[1], t[2] + s[2])
            else: new[k] = ('B',)
        st = new
        if not ch: break
        r_used = r + 1
    mb = sum(S[k][4] for k in range(N))
    byte_b = sum(S[k][4] for k in range(N) if st[k][0] in 'BP')
    nB = sum(1 for k in range(N) if st[k][0] in 'BP')
    print(f"{kind:10s} seed {seed}: seqs {N}, match bytes {mb}, piece rounds {r_used}, byte-level pieces {nB} ({100*nB/max(1,N):.1f} %), "
          f"their bytes {byte_b} ({100*byte_b/max(1,mb):.1f} % of match bytes)")

def final_runs(kind, seed):
    # the floor of any run-level scheme: maximal runs of consecutive literal sources in the resolved output
    src = O.generate(kind, seed, 4 << 20); S = parse(O.compress_block_bytes(src))
    n = src.size; ptr = np.empty(n, np.int64)
    for xs, ls, ll, off, ml in S:
        ptr[xs:xs + ll] = -1 - np.arange(ls, ls + ll)      # literal: -1 - compressed position
        if ml:
            ms = xs + ll; d = np.arange(ml)
            ptr[ms:ms + ml] = np.where(d < off, ms + d, ms + d % off) - off
    r = 0
    while (ptr >= 0).any():
        m = ptr >= 0; ptr[m] = ptr[ptr[m]]; r += 1
    brk = np.count_nonzero(np.diff(-1 - ptr) != 1) + 1
    print(f"{kind:10s} seed {seed}: {brk} runs of consecutive literal sources, mean run {n / brk:.1f} B, byte rounds {r}")


if __name__ == "__main__":
    for kind in sys.argv[1].split(','):
        for seed in (1, 2):
            model(kind, seed)
        final_runs(kind, 1)
