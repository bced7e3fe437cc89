/*
 * synth.c -- deterministic synthetic chromosome pairs for tests and bench.py (see synth.h).
 * The generator is sequential (xoshiro256** seeded by splitmix64 of the seed), so one seed gives
 * the same bytes on every machine.  ~1 s per 250 Mb pair.
 */
#include "synth.h"

#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s[4]; } rng_t;

static uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t* r, uint64_t seed) {
    uint64_t x = seed * 0x2545F4914F6CDD1Dull + 12345;
    for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&x);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rng_next(rng_t* r) {
    uint64_t* s = r->s;
    uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static inline double rng_u01(rng_t* r) { return (double)(rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline int64_t rng_range(rng_t* r, int64_t lo, int64_t hi) {   /* inclusive */
    return lo + (int64_t)(rng_next(r) % (uint64_t)(hi - lo + 1));
}
static const char BASES[4] = {'A', 'C', 'G', 'T'};
static inline char rbase(rng_t* r) { return BASES[rng_next(r) & 3]; }

typedef struct { char* d; int64_t n, cap; int oom; } vec_t;
static void vput(vec_t* v, char c) {
    if (v->oom) return;
    if (v->n == v->cap) {
        int64_t nc = v->cap ? v->cap * 2 : 4096;
        char* nd = (char*)realloc(v->d, (size_t)nc);
        if (!nd) { v->oom = 1; return; }
        v->d = nd; v->cap = nc;
    }
    v->d[v->n++] = c;
}

static char* to_fasta(const char* name, const char* s, int64_t n, size_t* out_n) {
    size_t hl = strlen(name);
    size_t cap = hl + 2 + (size_t)n + (size_t)(n / 50) + 2;
    char* f = (char*)malloc(cap);
    if (!f) return NULL;
    size_t w = 0;
    f[w++] = '>';
    memcpy(f + w, name, hl); w += hl;
    f[w++] = '\n';
    for (int64_t i = 0; i < n; i += 50) {
        int64_t c = n - i < 50 ? n - i : 50;
        memcpy(f + w, s + i, (size_t)c); w += (size_t)c;
        f[w++] = '\n';
    }
    *out_n = w;
    return f;
}

static inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }
static inline int is_lower(char c) { return c >= 'a' && c <= 'z'; }

int synth_pair(int profile, int64_t ref_len, int64_t tgt_len, uint64_t seed, const char* ref_name,
               const char* tgt_name, char** ref_fa, size_t* ref_n, char** tgt_fa, size_t* tgt_n) {
    rng_t r;
    rng_seed(&r, seed);
    int64_t n = ref_len;
    char* R = (char*)malloc((size_t)(n > 0 ? n : 1));
    if (!R) return 1;
    for (int64_t i = 0; i < n; i++) R[i] = rbase(&r);

    /* interspersed repeat family: 300-bp consensus, divergent copies + poly-A tail */
    {
        const int rl = 300, pa = 20;
        const double div = 0.10, cover = 0.10;
        char cons[300];
        for (int i = 0; i < rl; i++) cons[i] = rbase(&r);
        int64_t copies = (int64_t)(cover * (double)n / (rl + pa));
        for (int64_t c = 0; c < copies && n > rl + pa; c++) {
            int64_t at = rng_range(&r, 0, n - rl - pa);
            for (int i = 0; i < rl; i++) R[at + i] = rng_u01(&r) < div ? rbase(&r) : cons[i];
            for (int i = 0; i < pa; i++) R[at + rl + i] = 'A';
        }
    }
    /* T2T-like: Mb-scale 171-bp tandem arrays at 2-5 % divergence (scaled to the length) */
    if (profile == SYNTH_T2T && n > 20000) {
        char unit[171];
        for (int i = 0; i < 171; i++) unit[i] = rbase(&r);
        int arrays = 3;
        int64_t alen = n / 40;
        if (alen > 3000000) alen = 3000000;
        for (int a = 0; a < arrays; a++) {
            int64_t at = rng_range(&r, 0, n - alen);
            double dv = 0.02 + 0.03 * rng_u01(&r);
            for (int64_t i = 0; i < alen; i++) R[at + i] = rng_u01(&r) < dv ? rbase(&r) : unit[i % 171];
        }
    }
    /* soft-masking: runs of 50-1150 bases covering ~45 % */
    {
        int64_t p = 0;
        while (p < n) {
            p += rng_range(&r, 0, 1466);
            int64_t len = rng_range(&r, 50, 1150);
            for (int64_t i = p; i < p + len && i < n; i++) R[i] = lower(R[i]);
            p += len;
        }
    }
    /* N gaps: both ends + a centromeric gap */
    int64_t end_gap = n / 20 < 10000 ? n / 20 : 10000;
    int64_t cen = n >= 200000 ? n / 50 : 0, cen_at = n / 3;
    for (int64_t i = 0; i < end_gap; i++) { R[i] = 'N'; R[n - 1 - i] = 'N'; }
    for (int64_t i = 0; i < cen; i++) R[cen_at + i] = 'N';

    /* target = mutated reference */
    double snp = 1e-3, indel = 1e-4;
    int indel_max = 20, big_ins = 0, tgt_gaps = 1;
    int64_t big_del_every = 0;
    int64_t body = n - 2 * end_gap - cen;
    if (profile == SYNTH_HG) big_ins = body > 30000 ? 3 + (int)(body / 50000000) : (body > 6000 ? 1 : 0);
    if (profile == SYNTH_LOCAL) indel = 0;
    if (profile == SYNTH_T2T) { snp = 1e-2; big_del_every = 100000; tgt_gaps = 0; }
    int64_t ins_at[64];
    for (int i = 0; i < big_ins && i < 64; i++) ins_at[i] = rng_range(&r, end_gap + 1000, n - end_gap - 1000);
    vec_t T = {0};
    int64_t next_del = big_del_every ? rng_range(&r, big_del_every / 2, big_del_every) : -1;
    for (int64_t i = 0; i < n; i++) {
        char c = R[i];
        if (c == 'N') { vput(&T, tgt_gaps ? 'N' : rbase(&r)); continue; }
        for (int b = 0; b < big_ins; b++)
            if (ins_at[b] == i) {
                int64_t len = rng_range(&r, 1000, 5000);
                for (int64_t j = 0; j < len; j++) vput(&T, rbase(&r));
            }
        if (next_del >= 0 && i >= next_del) {
            i += rng_range(&r, 101, 500);
            next_del = i + rng_range(&r, big_del_every / 2, 3 * big_del_every / 2);
            continue;
        }
        double u = rng_u01(&r);
        if (u < snp) {
            char nb;
            do { nb = rbase(&r); } while (nb == (char)(c & ~32));
            vput(&T, is_lower(c) ? lower(nb) : nb);
        } else if (u < snp + indel) {
            int64_t len = rng_range(&r, 1, indel_max);
            if (rng_next(&r) & 1) {
                for (int64_t j = 0; j < len; j++) vput(&T, rbase(&r));
                vput(&T, c);
            } else {
                i += len - 1;
            }
        } else {
            vput(&T, c);
        }
    }
    /* exact target length: pad or trim just before the terminal N gap */
    {
        int64_t tail = 0;
        while (tail < T.n && T.d[T.n - 1 - tail] == 'N') tail++;
        int64_t want_body = tgt_len - tail;
        if (want_body < 0) want_body = 0;
        int64_t have_body = T.n - tail;
        char* tailbuf = (char*)malloc((size_t)(tail > 0 ? tail : 1));
        if (!tailbuf) { free(R); free(T.d); return 1; }
        memcpy(tailbuf, T.d + have_body, (size_t)tail);
        T.n = have_body < want_body ? have_body : want_body;
        while (T.n < want_body) vput(&T, rbase(&r));
        for (int64_t i = 0; i < tail && T.n < tgt_len; i++) vput(&T, tailbuf[i]);
        free(tailbuf);
    }
    if (T.oom) { free(R); free(T.d); return 1; }
    *ref_fa = to_fasta(ref_name, R, n, ref_n);
    *tgt_fa = to_fasta(tgt_name, T.d, T.n, tgt_n);
    free(R);
    free(T.d);
    return (*ref_fa && *tgt_fa) ? 0 : 1;
}

void synth_free(void* p) { free(p); }
