// tools/proto/segpar.c — CPU prototype of the exact segment-parallel LZ4 parse
// (design study for the GPU batch encoder; not product code).
//
// The reference parse (blockCompress.js:48-175) is one greedy chain, but a probe
// at i only uses a table entry q with i - q <= 65535. With 64 KiB segments,
// segment k's parse therefore depends only on (a) its entry state (first probe
// position, anchor, skip counter) and (b) the probes of segment k-1 (its "own"
// table). Every segment runs speculatively from a guess, logs each entry-table
// value it consumes, and is re-run (Jacobi) until every segment's entry state and
// consumed values equal what its predecessor's latest run provides. The result is
// the serial parse exactly. This prototype measures how many passes that takes.
//
//   gcc -O2 -o /tmp/segpar tools/proto/segpar.c && /tmp/segpar
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SEG 65536
#define NH 16384

static uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint32_t hsh(uint32_t s) { return (s * 2654435761u) >> 18; }

typedef struct { int32_t i, anchor; uint32_t c; } state_t;
typedef struct { int32_t pos, cand, end, anchor; } seqr_t;    // match at pos from cand, ends at end
typedef struct { uint16_t h; int32_t i, v; } logent_t;       // consumed entry: probe i read v (normalised)

typedef struct {
    int32_t own[NH];          // own probes of the latest run (-1 empty)
    int runs;
    state_t in, out;          // entry state used / exit state of the latest run
    logent_t* log; int nlog;
    seqr_t* seq; int nseq;
    int nprobe;
} seg_t;

// normalise a table value for probe i: out of range -> -1
static const uint8_t* g_src;
static int32_t norm(int32_t q, int32_t i) {
    if (q < 0 || q >= i || i - q > 65535) return -1;
    return rd32(g_src + q) == rd32(g_src + i) ? q : -1;     // outcome: hit with q, or miss
}

// Run segment k: entry state `st`, entry table `et` (values < k*SEG, -1 empty).
static void run(const uint8_t* src, int32_t n, int k, state_t st, const int32_t* et, seg_t* S, int32_t mflimit,
                int32_t matchlimit) {
    const int32_t lo = k * SEG, hi = (k + 1) * SEG;
    for (int h = 0; h < NH; ++h) S->own[h] = -1;
    static uint8_t touched[NH];
    memset(touched, 0, sizeof touched);
    S->nlog = 0; S->nseq = 0; S->nprobe = 0; S->in = st; S->runs++;
    int32_t i = st.i, anchor = st.anchor;
    uint32_t c = st.c;
    (void)lo;
    while (i < mflimit && i < hi) {
        uint32_t seq = rd32(src + i);
        uint32_t h = hsh(seq);
        int32_t cand;
        S->nprobe++;
        if (touched[h]) cand = S->own[h];
        else {
            cand = norm(et ? et[h] : -1, i);
            S->log[S->nlog++] = (logent_t){(uint16_t)h, i, cand};
            touched[h] = 1;
        }
        S->own[h] = i;
        if (cand < 0 || cand == i || i - cand > 65535 || rd32(src + cand) != seq) { i += c++ >> 6; continue; }
        c = 67;
        int32_t e = i + 4, m = cand + 4;
        while (e < matchlimit && src[e] == src[m]) { ++e; ++m; }
        S->seq[S->nseq++] = (seqr_t){i, cand, e, anchor};
        i = e; anchor = e;
    }
    S->out = (state_t){i, anchor, c};
    (void)n;
}

static int same_state(state_t a, state_t b) { return a.i == b.i && a.anchor == b.anchor && a.c == b.c; }

// serial reference parse, for verification
static int serial(const uint8_t* src, int32_t n, seqr_t* out) {
    static int32_t T[NH];
    for (int h = 0; h < NH; ++h) T[h] = -1;
    int32_t mflimit = n - 12, matchlimit = n - 5, i = 0, anchor = 0, ns = 0;
    uint32_t c = 67;
    while (i < mflimit) {
        uint32_t seq = rd32(src + i), h = hsh(seq);
        int32_t cand = T[h];
        T[h] = i;
        if (cand < 0 || cand == i || i - cand > 65535 || rd32(src + cand) != seq) { i += c++ >> 6; continue; }
        c = 67;
        int32_t e = i + 4, m = cand + 4;
        while (e < matchlimit && src[e] == src[m]) { ++e; ++m; }
        out[ns++] = (seqr_t){i, cand, e, anchor};
        i = e; anchor = e;
    }
    return ns;
}

static uint32_t xs(uint32_t* x) { *x ^= *x << 13; *x ^= *x >> 17; *x ^= *x << 5; return *x; }
static void gen(int kind, uint32_t seed, uint8_t* b, int n) {
    uint32_t x = seed ? seed : 1;
    if (kind == 0) { for (int i = 0; i < n; i += 4) { uint32_t v = xs(&x); for (int k = 0; k < 4 && i + k < n; ++k) b[i + k] = v >> (8 * k); } }
    else if (kind == 1) { for (int i = 0; i < n; ++i) b[i] = i % 251; }
    else if (kind == 2) {
        uint8_t t[216 * 64]; for (int k = 0; k < 216 * 64; ++k) t[k] = xs(&x) & 255;
        int i = 0; while (i < n) { int base = 64 * (xs(&x) % 216); for (int k = 0; k < 64 && i < n; ++k) b[i++] = t[base + k]; }
    } else if (kind == 3) {   // text-like words
        const char* w[] = {"the","of","and","to","in","is","was","for","on","that","with","as","by","at","from","his","an","were","are","which","this","be","or","has","had","not","but","it","its"};
        int i = 0; while (i < n) { uint32_t v = xs(&x); const char* s = w[v % 29]; for (int k = 0; s[k] && i < n; ++k) b[i++] = s[k]; if (i < n) b[i++] = ((v >> 16) % 11 == 0) ? 10 : 32; }
    } else {                  // copy generator
        int i = 0;
        while (i < n) {
            int L = 4 + xs(&x) % 5; for (int k = 0; k < L && i < n; ++k) b[i++] = xs(&x) & 255;
            int M = 48 + xs(&x) % 33, off = 16 + xs(&x) % 4081; if (i - off < 0) continue;
            for (int k = 0; k < M && i < n; ++k, ++i) b[i] = b[i - off];
        }
    }
}

int main(int argc, char** argv) {
    const int n = 4 << 20, nseg = n / SEG;
    int warm = argc > 1 ? atoi(argv[1]) : 1;        // warm-up segments before each segment in pass 0
    uint8_t* src = malloc(n);
    seqr_t* ref = malloc(sizeof(seqr_t) * (n / 4));
    seg_t* S = calloc(nseg, sizeof(seg_t));
    for (int k = 0; k < nseg; ++k) { S[k].log = malloc(sizeof(logent_t) * SEG); S[k].seq = malloc(sizeof(seqr_t) * SEG); }
    int32_t* warmT = malloc(sizeof(int32_t) * NH);
    const char* names[] = {"random", "repetitive", "tiles216", "text", "copy"};
    for (int kind = 0; kind < 5; ++kind) for (uint32_t seed = 1; seed <= 4; ++seed) {
        gen(kind, seed, src, n);
        g_src = src;
        int nref = serial(src, n, ref);
        int32_t mflimit = n - 12, matchlimit = n - 5;
        long probes0 = 0, probes = 0;
        // pass 0: each segment from its start, entry table from a warm-up over the previous `warm` segments
        for (int k = 0; k < nseg; ++k) {
            S[k].runs = 0;
            state_t st = {k * SEG, k * SEG, 67};
            int32_t* et = NULL;
            if (k > 0 && warm > 0) {
                static seg_t W; if (!W.log) { W.log = malloc(sizeof(logent_t) * SEG * 4); W.seq = malloc(sizeof(seqr_t) * SEG * 4); }
                int k0 = k - warm < 0 ? 0 : k - warm;
                state_t ws = {k0 * SEG, k0 * SEG, 67};
                // warm-up: run consecutive segments k0..k-1 chained, keep the last one's own table merged
                for (int h = 0; h < NH; ++h) warmT[h] = -1;
                int32_t* prevT = NULL;
                static int32_t tmp[NH];
                for (int w = k0; w < k; ++w) {
                    run(src, n, w, ws, prevT, &W, mflimit, matchlimit);
                    probes0 += W.nprobe;
                    memcpy(tmp, W.own, sizeof tmp);
                    prevT = tmp;
                    ws = W.out;
                }
                memcpy(warmT, tmp, sizeof tmp);
                et = warmT;
                if (ws.i >= k * SEG) st = ws;
            }
            run(src, n, k, st, et, &S[k], mflimit, matchlimit);
            probes0 += S[k].nprobe;
        }
        // serial sweep: with segment k-1 exact, segment k's pass-0 run is kept if its entry
        // position/skip state and every consumed outcome agree with k-1's exact run, else re-run
        int sweep_reruns = 0; long sweep_checks = 0, sweep_probes = 0;
        {
            static seg_t X[1024];
            static int init = 0;
            if (!init) { for (int k = 0; k < 1024; ++k) { X[k].log = malloc(sizeof(logent_t) * SEG); X[k].seq = malloc(sizeof(seqr_t) * SEG); } init = 1; }
            for (int k = 0; k < nseg; ++k) {
                if (k == 0) { memcpy(X[0].own, S[0].own, sizeof(S[0].own)); X[0].out = S[0].out; continue; }
                state_t want = X[k - 1].out;
                int ok = S[k].in.i == want.i && S[k].in.c == want.c;
                for (int e = 0; ok && e < S[k].nlog; ++e) {
                    sweep_checks++;
                    if (norm(X[k - 1].own[S[k].log[e].h], S[k].log[e].i) != S[k].log[e].v) ok = 0;
                }
                if (ok) { memcpy(X[k].own, S[k].own, sizeof(S[k].own)); X[k].out = S[k].out; }
                else { run(src, n, k, want, X[k - 1].own, &X[k], mflimit, matchlimit); sweep_reruns++; sweep_probes += X[k].nprobe; }
            }
        }
        printf("   sweep: reruns %d / %d, checks %ld, rerun probes %ld\n", sweep_reruns, nseg, sweep_checks, sweep_probes);
        // Jacobi passes: segment k is settled when its entry state == S[k-1].out and every
        // consumed value == normalised S[k-1].own
        int passes = 0, reruns = 0, why_state = 0, why_c = 0, why_log = 0;
        static int32_t snap[1024][NH];      // tables of the previous pass (Jacobi)
        static state_t snapst[1024];
        for (;;) {
            for (int k = 0; k < nseg; ++k) { memcpy(snap[k], S[k].own, sizeof(int32_t) * NH); snapst[k] = S[k].out; }
            int changed = 0;
            for (int k = 1; k < nseg; ++k) {
                state_t want = snapst[k - 1];
                if (want.i < k * SEG) want = (state_t){k * SEG, want.anchor, want.c};   // cannot happen
                int ok = S[k].in.i == want.i && (S[k].in.c == want.c || (S[k].in.c < 128 && want.c < 128 && 0));
                if (!ok) { if (S[k].in.i != want.i) why_state++; else why_c++; }
                for (int e = 0; ok && e < S[k].nlog; ++e)
                    if (norm(snap[k - 1][S[k].log[e].h], S[k].log[e].i) != S[k].log[e].v) { ok = 0; why_log++; }
                if (!ok) { run(src, n, k, want, snap[k - 1], &S[k], mflimit, matchlimit); changed++; probes += S[k].nprobe; }
            }
            if (!changed) break;
            passes++; reruns += changed;
        }
        // verify
        int ns = 0, bad = 0;
        for (int k = 0; k < nseg; ++k) for (int q = 0; q < S[k].nseq; ++q) {
            if (ns >= nref || memcmp(&S[k].seq[q], &ref[ns], sizeof(seqr_t))) bad = 1;
            ns++;
        }
        printf("%-10s seed %u warm %d: seqs %7d  passes %2d  reruns %4d  why: pos %d c %d log %d  %s\n",
               names[kind], seed, warm, nref, passes, reruns, why_state, why_c, why_log,
               (bad || ns != nref) ? "MISMATCH" : "exact");
    }
    return 0;
}
