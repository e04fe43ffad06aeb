/* CPU model of a segment-parallel exact compressBlock parse (blockCompress.js:48-175).
 * Segment k covers [B_k, B_k+1); its speculative parse starts W bytes earlier with an empty table
 * and the skip counter at 67. The parse from a position on depends only on (next probe position,
 * skip counter, probed positions in the 65535 bytes before it), so a segment whose speculative
 * state at B_k equals the true one -- same next probe, same counter, same probes in
 * [B_k - 65535, B_k) -- is exact from there. Reports the share of segments certified.
 *   gcc -O2 -o /tmp/segcomp tools/proto/segcomp_model.c && /tmp/segcomp */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t xs(uint32_t* x) { *x ^= *x << 13; *x ^= *x >> 17; *x ^= *x << 5; return *x; }
static void gen(int kind, uint32_t seed, uint8_t* b, int n) {
    uint32_t r = seed ? seed : 1; int i = 0;
    if (kind == 0) { for (i = 0; i < n; i += 4) { uint32_t v = xs(&r); for (int k = 0; k < 4 && i + k < n; k++) b[i + k] = v >> (8 * k); } }
    else if (kind == 1) { for (i = 0; i < n; i++) b[i] = i % 251; }
    else if (kind == 2) { uint8_t t[216 * 64]; for (int k = 0; k < 216 * 64; k++) t[k] = xs(&r) & 255;
        while (i < n) { int base = 64 * (xs(&r) % 216); for (int k = 0; k < 64 && i < n; k++) b[i++] = t[base + k]; } }
    else if (kind == 3) { while (i < n) { int L = 4 + xs(&r) % 5; for (int k = 0; k < L && i < n; k++) b[i++] = xs(&r) & 255;
        int M = 48 + xs(&r) % 33, off = 16 + xs(&r) % 4081; if (i - off < 0) continue; for (int k = 0; k < M && i < n; k++, i++) b[i] = b[i - off]; } }
    else if (kind == 5) { const char* w[] = {"the","of","and","to","in","is","was","for","on","that","with","as","by","at","from","his","an","were","are","which","this","be","or","has","had","not","but","it","its"};
        while (i < n) { uint32_t v = xs(&r); const char* s = w[v % 29]; for (int k = 0; s[k] && i < n; k++) b[i++] = s[k]; if (i < n) b[i++] = ((v >> 16) % 11 == 0) ? 10 : 32; } }
}
static uint32_t rd32(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

/* parse from i0 (anchor irrelevant) with table T, counter m; stop at the first probe >= stop.
 * probes: bitmap of probed positions (absolute). returns next probe pos, *mo = counter there */
static int parse(const uint8_t* src, int n, int i0, uint32_t m, int32_t* T, uint8_t* probes, int stop, uint32_t* mo, long* nprobe) {
    const int mflimit = n - 12, matchlimit = n - 5;
    int i = i0;
    while (i < mflimit && i < stop) {
        uint32_t seq = rd32(src + i), h = (seq * 2654435761u) >> 18;
        int32_t cand = T[h] - 1; T[h] = i + 1;
        if (probes) probes[i >> 3] |= 1 << (i & 7);
        ++*nprobe;
        if (cand < 0 || cand == i || ((uint32_t)(i - cand) >> 16) || rd32(src + cand) != seq) { i += m++ >> 6; continue; }
        m = 67;
        int e = i + 4, c = cand + 4;
        while (e < matchlimit && src[e] == src[c]) { e++; c++; }
        i = e;
    }
    *mo = m;
    return i;
}

int main(int argc, char** argv) {
    const int n = 4 << 20;
    uint8_t* src = malloc(n);
    uint8_t* ptrue = malloc(n / 8 + 1);
    uint8_t* pspec = malloc(n / 8 + 1);
    int32_t* T = malloc(16384 * 4);
    const char* names[] = {"random", "repetitive", "tiles216", "copy", "runs", "text"};
    int kinds[] = {2, 5, 3, 0, 1};
    int Ls[] = {65536, 131072, 262144};
    int Ws[] = {65536 + 4096, 65536 + 16384, 65536 + 65536};
    for (int ki = 0; ki < 5; ki++) for (int seed = 1; seed <= 4; seed++) {
        int kind = kinds[ki];
        gen(kind, seed, src, n);
        /* true parse: states at every 64 KiB boundary */
        memset(ptrue, 0, n / 8 + 1); memset(T, 0, 16384 * 4);
        int nb = n / 65536; int bi[65]; uint32_t bm[65];
        int i = 0; uint32_t m = 67; long np = 0;
        for (int k = 1; k <= nb; k++) { i = parse(src, n, i, m, T, ptrue, k * 65536, &m, &np); bi[k] = i; bm[k] = m; }
        long np_true = np;
        for (int li = 0; li < 3; li++) for (int wi = 0; wi < 3; wi++) {
            int L = Ls[li], W = Ws[wi], S = n / L, ok = 0; long npw = 0;
            for (int k = 1; k < S; k++) {
                int B = k * L, s0 = B - W < 0 ? 0 : B - W;
                memset(pspec + (s0 >> 3), 0, (B >> 3) - (s0 >> 3) + 1); memset(T, 0, 16384 * 4);
                uint32_t ms; long q = 0;
                int is = parse(src, n, s0, 67, T, pspec, B, &ms, &q);
                npw += q;
                int good = is == bi[B / 65536] && ms == bm[B / 65536];
                for (int b = (B - 65536) >> 3; good && b < (B >> 3); b++) if (pspec[b] != ptrue[b]) good = 0;
                ok += good;
            }
            printf("%-9s seed %d  L=%4dK W=%3dK: certified %3d / %3d   warm-up probes %.2fx the block's\n", names[kind], seed,
                   L >> 10, W >> 10, ok, S - 1, (double)npw / np_true);
        }
    }
    return 0;
}
