/*
 * sccg_oracle.c -- CPU restatement of SCCG's compression/decompression path.
 *
 * TEST INFRASTRUCTURE ONLY: the parity oracle for the MI355X implementation.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load or run this file's
 * library; the product never links it.  Written from SURVEY.md Appendix A and a reading of
 * the reference; every function cites the reference lines it restates.
 *
 * Parity is pinned against the reference itself: oracle/_ref (the reference sources compiled
 * unchanged by `make -C oracle ref`) produced the fixtures in tests/golden/ with
 * tests/golden/make_golden.py, and tests/test_oracle_golden.py checks this file against them.
 *
 * Data-structure note: the reference keys an unordered_map<string_view, vector<int>> by the
 * k-mer bytes (compression.cpp:41-47); each vector holds ascending positions.  Here the same
 * "k-mer -> ascending positions" relation is a sorted array (radix-sorted 2-bit codes for pure
 * A/C/G/T k-mers, memcmp-sorted positions for k-mers holding any other byte).  Output depends
 * only on the per-key ascending order, never on hash iteration order.
 */
#define _GNU_SOURCE
#include "sccg_oracle.h"

#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* growable byte buffer                                                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    char* d;
    size_t n, cap;
    int oom;
} sb_t;

static void sb_reserve(sb_t* b, size_t extra) {
    if (b->oom) return;
    if (b->n + extra + 1 <= b->cap) return;
    size_t nc = b->cap ? b->cap : 256;
    while (nc < b->n + extra + 1) nc *= 2;
    char* nd = (char*)realloc(b->d, nc);
    if (!nd) { b->oom = 1; return; }
    b->d = nd;
    b->cap = nc;
}
static void sb_put(sb_t* b, const char* s, size_t n) {
    if (!n && b->d) return;
    sb_reserve(b, n);
    if (b->oom) return;
    if (n) memcpy(b->d + b->n, s, n);
    b->n += n;
    b->d[b->n] = 0;
}
static void sb_putc(sb_t* b, char c) { sb_put(b, &c, 1); }
static void sb_int(sb_t* b, long long v) {
    char tmp[32];
    int n = snprintf(tmp, sizeof tmp, "%lld", v);
    sb_put(b, tmp, (size_t)n);
}

/* C-locale ctype predicates used by the reference (::isspace, islower, toupper, tolower). */
static inline int c_isspace(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
static inline int c_islower(unsigned char c) { return c >= 'a' && c <= 'z'; }
static inline char c_toupper(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }
static inline char c_tolower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

/* ------------------------------------------------------------------------------------------ */
/* FASTA ingest -- compression.cpp:181-220 (also decompression.cpp:47-58 for the reference)    */
/* ------------------------------------------------------------------------------------------ */
/* Reference: every line that is non-empty and does not start with '>' is appended; then all
 * isspace bytes are erased (compression.cpp:193-200).  Lines split on '\n' only (getline). */
static void ingest_reference(const char* fa, size_t n, sb_t* out) {
    size_t i = 0;
    while (i < n) {
        size_t e = i;
        while (e < n && fa[e] != '\n') e++;
        if (e > i && fa[i] != '>') {
            for (size_t j = i; j < e; j++)
                if (!c_isspace((unsigned char)fa[j])) sb_putc(out, fa[j]);
        }
        i = e + 1;
    }
}

/* Target: the FIRST line starting with '>' is the header; every other non-empty line
 * (including later '>' lines) is sequence; then isspace erased (compression.cpp:207-218). */
static void ingest_target(const char* fa, size_t n, sb_t* out, sb_t* header, int* has_header) {
    size_t i = 0;
    *has_header = 0;
    while (i < n) {
        size_t e = i;
        while (e < n && fa[e] != '\n') e++;
        if (e > i) {
            if (!*has_header && fa[i] == '>') {
                sb_put(header, fa + i, e - i);
                *has_header = 1;
            } else {
                for (size_t j = i; j < e; j++)
                    if (!c_isspace((unsigned char)fa[j])) sb_putc(out, fa[j]);
            }
        }
        i = e + 1;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* k-mer -> ascending positions (the relation of compression.cpp:41-47)                        */
/* ------------------------------------------------------------------------------------------ */
static inline int base2(unsigned char c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

typedef struct {
    uint64_t code;
    int32_t pos;
} kpos_t;

typedef struct {
    int k;
    const char* s;
    int64_t n;            /* |Sr| */
    uint64_t* pure;       /* k <= 16: (code << 32) | pos, sorted by code then pos */
    kpos_t* pure2;        /* k > 16 (parameter overrides): (code, pos), sorted the same way */
    int64_t npure;
    int32_t* exo;         /* positions of k-mers holding a non-ACGT byte, sorted by bytes then pos */
    int64_t nexo;
} kindex_t;

static __thread const char* g_cmp_s;
static __thread int g_cmp_k;
static int cmp_exo(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    int c = memcmp(g_cmp_s + x, g_cmp_s + y, (size_t)g_cmp_k);
    if (c) return c;
    return (x > y) - (x < y);
}
static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}
static int cmp_kpos(const void* a, const void* b) {
    const kpos_t* x = (const kpos_t*)a;
    const kpos_t* y = (const kpos_t*)b;
    if (x->code != y->code) return (x->code > y->code) - (x->code < y->code);
    return (x->pos > y->pos) - (x->pos < y->pos);
}

static void radix_sort_u64_hi(uint64_t* a, int64_t n, int bits) {
    /* stable LSD over bits [32, 32+bits) -- input positions ascending, so output is sorted by
     * (code, pos) */
    uint64_t* tmp = (uint64_t*)malloc((size_t)n * sizeof(uint64_t));
    if (!tmp) { qsort(a, (size_t)n, sizeof(uint64_t), cmp_u64); return; }
    const int D = 11;
    size_t cnt[1 << D];
    for (int sh = 32; sh < 32 + bits; sh += D) {
        memset(cnt, 0, sizeof cnt);
        for (int64_t i = 0; i < n; i++) cnt[(a[i] >> sh) & ((1u << D) - 1)]++;
        size_t s = 0;
        for (int d = 0; d < (1 << D); d++) { size_t c = cnt[d]; cnt[d] = s; s += c; }
        for (int64_t i = 0; i < n; i++) tmp[cnt[(a[i] >> sh) & ((1u << D) - 1)]++] = a[i];
        uint64_t* t = a; a = tmp; tmp = t;
        /* after an odd number of passes the data lives in the other buffer */
    }
    int passes = (bits + D - 1) / D;
    if (passes & 1) { memcpy(tmp, a, (size_t)n * sizeof(uint64_t)); free(a); }
    else free(tmp);
}

static int kindex_build(kindex_t* ix, const char* s, int64_t n, int k) {
    memset(ix, 0, sizeof *ix);
    ix->k = k; ix->s = s; ix->n = n;
    if (n < k) return ORC_OK;   /* H stays empty (compression.cpp:44 loop never runs) */
    int64_t nk = n - k + 1;
    const int wide = k > 16;   /* 2k-bit codes no longer fit beside a 32-bit position */
    if (wide) ix->pure2 = (kpos_t*)malloc((size_t)nk * sizeof(kpos_t));
    else ix->pure = (uint64_t*)malloc((size_t)nk * sizeof(uint64_t));
    ix->exo = (int32_t*)malloc((size_t)nk * sizeof(int32_t));
    if ((!ix->pure && !ix->pure2) || !ix->exo) return ORC_E_ALLOC;
    uint64_t mask = (k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    uint64_t code = 0;
    int64_t last_bad = -1;
    for (int64_t i = 0; i < n; i++) {
        int b = base2((unsigned char)s[i]);
        if (b < 0) { last_bad = i; b = 0; }
        code = ((code << 2) | (uint64_t)b) & mask;
        int64_t st = i - k + 1;
        if (st < 0) continue;
        if (last_bad >= st) ix->exo[ix->nexo++] = (int32_t)st;
        else if (wide) { ix->pure2[ix->npure].code = code; ix->pure2[ix->npure++].pos = (int32_t)st; }
        else ix->pure[ix->npure++] = (code << 32) | (uint64_t)st;
    }
    if (ix->npure > 1) {   /* (the arrays may be NULL when empty) */
        if (wide) qsort(ix->pure2, (size_t)ix->npure, sizeof(kpos_t), cmp_kpos);
        else if (ix->npure < 4096) qsort(ix->pure, (size_t)ix->npure, sizeof(uint64_t), cmp_u64);
        else radix_sort_u64_hi(ix->pure, ix->npure, 2 * k);
    }
    g_cmp_s = s; g_cmp_k = k;
    if (ix->nexo > 1) qsort(ix->exo, (size_t)ix->nexo, sizeof(int32_t), cmp_exo);
    return ORC_OK;
}

static void kindex_free(kindex_t* ix) {
    free(ix->pure);
    free(ix->pure2);
    free(ix->exo);
    memset(ix, 0, sizeof *ix);
}

/* Candidate range for the k bytes at q.  *pure_mode tells which array [lo,hi) indexes. */
static void kindex_lookup(const kindex_t* ix, const char* q, int64_t* lo, int64_t* hi, int* pure_mode) {
    int k = ix->k;
    uint64_t code = 0;
    int pure = 1;
    for (int j = 0; j < k; j++) {
        int b = base2((unsigned char)q[j]);
        if (b < 0) { pure = 0; break; }
        code = (code << 2) | (uint64_t)b;
    }
    *pure_mode = pure;
    if (pure && ix->pure2) {
        *pure_mode = 2;
        int64_t a = 0, z = ix->npure;
        while (a < z) { int64_t mid = (a + z) / 2; if (ix->pure2[mid].code < code) a = mid + 1; else z = mid; }
        *lo = a;
        z = ix->npure;
        while (a < z) { int64_t mid = (a + z) / 2; if (ix->pure2[mid].code <= code) a = mid + 1; else z = mid; }
        *hi = a;
    } else if (pure) {
        int64_t a = 0, z = ix->npure;
        while (a < z) { int64_t mid = (a + z) / 2; if ((ix->pure[mid] >> 32) < code) a = mid + 1; else z = mid; }
        *lo = a;
        z = ix->npure;
        while (a < z) { int64_t mid = (a + z) / 2; if ((ix->pure[mid] >> 32) <= code) a = mid + 1; else z = mid; }
        *hi = a;
    } else {
        int64_t a = 0, z = ix->nexo;
        while (a < z) { int64_t mid = (a + z) / 2; if (memcmp(ix->s + ix->exo[mid], q, (size_t)k) < 0) a = mid + 1; else z = mid; }
        *lo = a;
        z = ix->nexo;
        while (a < z) { int64_t mid = (a + z) / 2; if (memcmp(ix->s + ix->exo[mid], q, (size_t)k) <= 0) a = mid + 1; else z = mid; }
        *hi = a;
    }
}

static inline int32_t kindex_pos(const kindex_t* ix, int pure_mode, int64_t j) {
    return pure_mode == 2 ? ix->pure2[j].pos : pure_mode ? (int32_t)(ix->pure[j] & 0xffffffffu) : ix->exo[j];
}

/* ------------------------------------------------------------------------------------------ */
/* match_sequences -- compression.cpp:27-34 (extend_alignment) and :36-179                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    orc_rec* r;
    int64_t n, cap;
    int oom;
} recv_t;

static void rec_push(recv_t* v, int kind, int32_t p, int32_t l, int64_t t) {
    if (v->oom) return;
    if (v->n == v->cap) {
        int64_t nc = v->cap ? v->cap * 2 : 64;
        orc_rec* nr = (orc_rec*)realloc(v->r, (size_t)nc * sizeof(orc_rec));
        if (!nr) { v->oom = 1; return; }
        v->r = nr; v->cap = nc;
    }
    v->r[v->n].kind = kind; v->r[v->n].p = p; v->r[v->n].l = l; v->r[v->n].t = t;
    v->n++;
}

static inline int iabs(int x) { return x < 0 ? -x : x; }

/* compression.cpp:27-34: grow l from k while both strings continue and bytes agree. */
static inline int extend_len(const char* sr, int nr, const char* st, int nt, int p, int idx, int k) {
    int l = k;
    while (p + l < nr && idx + l < nt && sr[p + l] == st[idx + l]) ++l;
    return l;
}

static int match_core(const kindex_t* H, const char* sr, int nr, const char* st, int nt, int k,
                      int m, int global, int offset, recv_t* out) {
    int index = 0, pme = -1;
    int64_t lit_t = -1, lit_n = 0;   /* the open literal run is always St[lit_t, lit_t+lit_n) */
    while (index < nt - k + 1) {                                   /* :64 */
        int64_t lo, hi; int pm;
        kindex_lookup(H, st + index, &lo, &hi, &pm);                /* :75-77 */
        int take_literal = (lo == hi);
        if (!take_literal && global) {                             /* :83-96 range gate */
            int in_range = 0;
            for (int64_t j = lo; j < hi; j++) {
                int p = kindex_pos(H, pm, j);
                if (pme == -1 || iabs(p - pme) <= m) { in_range = 1; break; }
            }
            take_literal = !in_range;
        }
        if (take_literal) {
            if (lit_n == 0) lit_t = index;
            lit_n++;
            index++;
            continue;
        }
        if (lit_n) { rec_push(out, 0, 0, (int32_t)lit_n, lit_t); lit_n = 0; }  /* :97-107 */
        /* candidate selection, candidates visited in ascending order (:110-130) */
        int lmax1 = 0, lmax2 = 0, pn1 = 0, pn2 = 0, ln1 = 0, ln2 = 0;
        for (int64_t j = lo; j < hi; j++) {
            int p = kindex_pos(H, pm, j);
            int l = extend_len(sr, nr, st, nt, p, index, k);
            if (global && (pme == -1 || iabs(p - pme) <= m)) {
                if (l == lmax2) {
                    if (pn2 == 0 || iabs(p - pme) < iabs(pn2 - pme)) pn2 = p;
                } else if (l > lmax2) {
                    lmax2 = l; pn2 = p; ln2 = l;
                }
            }
            if (l == lmax1) {
                if (pn1 == 0 || iabs(p - pme) < iabs(pn1 - pme)) pn1 = p;
            } else if (l > lmax1) {
                lmax1 = l; pn1 = p; ln1 = l;
            }
        }
        int fp, fl;
        if (global && pn2 != 0) { fp = pn2; fl = ln2; }              /* :134-138 */
        else { fp = pn1; fl = ln1; }
        pme = fp + fl - 1;                                          /* :149 */
        rec_push(out, 1, fp + offset, fl, index);                   /* :152-156 */
        index += fl;                                                /* :159 */
    }
    if (index < nt) {                                               /* :164-167 */
        if (lit_n == 0) lit_t = index;
        lit_n += nt - index;
    }
    if (lit_n) rec_push(out, 0, 0, (int32_t)lit_n, lit_t);
    return out->oom ? ORC_E_ALLOC : ORC_OK;
}

/* The global walk of match_core (compression.cpp:64-161, global = 1) from an arbitrary state
 * (index = x0, prev_match_end = P0) up to the first state with index >= x_end: its match records
 * (kind 1, t = target index; literals are the gaps) and that exit state.  Two walks that reach the
 * same (index, P) are identical afterwards -- the property the chunked GPU walk and the
 * cross-GPU split of one chromosome rest on.  TEST INFRASTRUCTURE ONLY. */
int orc_walk_range(const char* sr, int64_t nr, const char* st, int64_t nt, int k, int m, int64_t x0, int64_t P0,
                   int64_t x_end, orc_rec** recs, int64_t* nrec, int64_t* exit_x, int64_t* exit_P) {
    kindex_t H;
    recv_t v = {0};
    int rc = kindex_build(&H, sr, nr, k);
    if (rc != ORC_OK) { *recs = NULL; *nrec = 0; return rc; }
    int index = (int)x0, pme = (int)P0;
    const int ntk = (int)nt - k + 1;
    while (index < ntk && index < x_end) {
        int64_t lo, hi; int pm;
        kindex_lookup(&H, st + index, &lo, &hi, &pm);
        int take_literal = (lo == hi);
        if (!take_literal) {
            int in_range = 0;
            for (int64_t j = lo; j < hi; j++) {
                int p = kindex_pos(&H, pm, j);
                if (pme == -1 || iabs(p - pme) <= m) { in_range = 1; break; }
            }
            take_literal = !in_range;
        }
        if (take_literal) { index++; continue; }
        int lmax1 = 0, lmax2 = 0, pn1 = 0, pn2 = 0, ln1 = 0, ln2 = 0;
        for (int64_t j = lo; j < hi; j++) {
            int p = kindex_pos(&H, pm, j);
            int l = extend_len(sr, (int)nr, st, (int)nt, p, index, k);
            if (pme == -1 || iabs(p - pme) <= m) {
                if (l == lmax2) {
                    if (pn2 == 0 || iabs(p - pme) < iabs(pn2 - pme)) pn2 = p;
                } else if (l > lmax2) {
                    lmax2 = l; pn2 = p; ln2 = l;
                }
            }
            if (l == lmax1) {
                if (pn1 == 0 || iabs(p - pme) < iabs(pn1 - pme)) pn1 = p;
            } else if (l > lmax1) {
                lmax1 = l; pn1 = p; ln1 = l;
            }
        }
        int fp, fl;
        if (pn2 != 0) { fp = pn2; fl = ln2; }
        else { fp = pn1; fl = ln1; }
        pme = fp + fl - 1;
        rec_push(&v, 1, fp, fl, index);
        index += fl;
    }
    kindex_free(&H);
    if (v.oom) { free(v.r); *recs = NULL; *nrec = 0; return ORC_E_ALLOC; }
    *recs = v.r;
    *nrec = v.n;
    *exit_x = index;   /* >= x_end, or the walk ran out of k-mers (index >= |St| - k + 1) */
    *exit_P = pme;
    return ORC_OK;
}

int orc_match(const char* sr, int64_t nr, const char* st, int64_t nt, int k, int m, int global,
              int64_t offset, orc_rec** recs, int64_t* nrec) {
    kindex_t H;
    recv_t v = {0};
    int rc = kindex_build(&H, sr, nr, k);
    if (rc == ORC_OK) rc = match_core(&H, sr, (int)nr, st, (int)nt, k, m, global, (int)offset, &v);
    kindex_free(&H);
    if (rc != ORC_OK) { free(v.r); *recs = NULL; *nrec = 0; return rc; }
    *recs = v.r;
    *nrec = v.n;
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* run lines: lowercase (compression.cpp:341-368, :495-522) and N (:527-555)                  */
/* ------------------------------------------------------------------------------------------ */
/* A run of length 1 prints "delta," ; longer runs "(delta,len)"; a run still open at the end of
 * the sequence prints "delta" (no comma) or "(delta,len)".  delta is against the previous run
 * start, which begins at 0. */
static void emit_run(sb_t* b, int delta, int len, int at_end) {
    if (len == 1) {
        sb_int(b, delta);
        if (!at_end) sb_putc(b, ',');
    } else {
        sb_putc(b, '(');
        sb_int(b, delta);
        sb_putc(b, ',');
        sb_int(b, len);
        sb_putc(b, ')');
    }
}

static void run_line(sb_t* b, const char* s, int64_t n, int which /*0 lower, 1 'N'*/) {
    int prev = 0;
    int64_t start = -1, len = 0;
    for (int64_t i = 0; i < n; i++) {
        int hit = which ? (s[i] == 'N') : c_islower((unsigned char)s[i]);
        if (hit) {
            if (len == 0) start = i;
            len++;
        } else if (len) {
            emit_run(b, (int)(start - prev), (int)len, 0);
            prev = (int)start;
            len = 0;
        }
    }
    if (len) emit_run(b, (int)(start - prev), (int)len, 1);
}

/* ------------------------------------------------------------------------------------------ */
/* delta_encode -- compression.cpp:222-304, restated as one linear pass                       */
/* ------------------------------------------------------------------------------------------ */
/* std::stoi on a substring: strtol semantics on its c_str(); throws when nothing converts or
 * the value leaves int.  Returns 0 on success. */
static int stoi_like(const char* s, size_t n, int* out) {
    char stackbuf[64];
    char* tmp = n < sizeof stackbuf ? stackbuf : (char*)malloc(n + 1);
    if (!tmp) return -1;
    memcpy(tmp, s, n);
    tmp[n] = 0;
    char* end = NULL;
    errno = 0;
    long v = strtol(tmp, &end, 10);
    int bad = (end == tmp) || errno == ERANGE || v > INT_MAX || v < INT_MIN;
    if (tmp != stackbuf) free(tmp);
    if (bad) return -1;
    *out = (int)v;
    return 0;
}

static const char* memchr_from(const char* s, size_t n, size_t from, char c) {
    if (from >= n) return NULL;
    return (const char*)memchr(s + from, c, n - from);
}

static int delta_encode(const char* s, size_t n, sb_t* out) {
    size_t search_start = 0;
    /* :236-256 -- skip the header/lowercase/N lines (3 newlines with a header, else 2) */
    int want = (n > 0 && s[0] == '>') ? 3 : 2;
    {
        size_t p = 0; int found = 0;
        const char* nl;
        while (found < want && (nl = memchr_from(s, n, p, '\n')) != NULL) {
            p = (size_t)(nl - s) + 1; found++;
        }
        if (found == want) search_start = p;
    }
    sb_put(out, s, search_start);
    size_t pos = search_start;
    int prev = 0;
    for (;;) {                                                      /* :262-293 */
        const char* op = memchr_from(s, n, pos, '(');
        if (!op) break;
        size_t open = (size_t)(op - s);
        const char* cp = memchr_from(s, n, open + 1, ')');
        if (!cp) break;
        size_t close = (size_t)(cp - s);
        const char* tok = s + open + 1;
        size_t tn = close - open - 1;
        const char* comma = (const char*)memchr(tok, ',', tn);
        if (!comma) {                                               /* :274-277 */
            sb_put(out, s + pos, close + 1 - pos);
            pos = close + 1;
            continue;
        }
        int start_ref;
        if (stoi_like(tok, (size_t)(comma - tok), &start_ref)) return ORC_E_DELTA_STOI;
        int delta = (int)((unsigned)start_ref - (unsigned)prev);    /* :280 (two's complement) */
        prev = start_ref;
        sb_put(out, s + pos, open + 1 - pos);
        sb_int(out, delta);
        sb_put(out, comma, (size_t)(s + close - comma));           /* ",len" -- :284 */
        pos = close;                                                /* :292 lands on ')' */
    }
    sb_put(out, s + pos, n - pos);
    return out->oom ? ORC_E_ALLOC : ORC_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* compress_genome -- compression.cpp:320-582 (without the 7z call at :581)                   */
/* ------------------------------------------------------------------------------------------ */
static __thread int g_last_global;
static __thread int64_t g_last_switch;
int orc_last_mode_global(void) { return g_last_global; }
int64_t orc_last_switch_segment(void) { return g_last_switch; }

static int emit_records(sb_t* f, const orc_rec* r, int64_t n, const char* st, int64_t* lit_bytes) {
    int64_t lit = 0;
    for (int64_t j = 0; j < n; j++) {
        if (r[j].kind) {
            sb_putc(f, '(');
            sb_int(f, r[j].p);
            sb_putc(f, ',');
            sb_int(f, r[j].l);
            sb_putc(f, ')');
        } else {
            sb_put(f, st + r[j].t, (size_t)r[j].l);
            lit += r[j].l;
        }
    }
    if (lit_bytes) *lit_bytes = lit;
    return f->oom ? ORC_E_ALLOC : ORC_OK;
}

static int has_non_n(const char* s, int64_t n) {
    for (int64_t i = 0; i < n; i++) if (s[i] != 'N') return 1;
    return 0;
}

/* any match record?  (compression.cpp:402 / :429 success test) */
static int any_match(const orc_rec* r, int64_t n) {
    for (int64_t j = 0; j < n; j++) if (r[j].kind) return 1;
    return 0;
}

void orc_params_default(orc_params* p) {
    p->k = 14; p->k2 = 10; p->L = 1000; p->m = 100; p->T1 = 0.5f; p->T2 = 4; p->local = 1;   /* :373-379 */
}

int orc_compress(const char* ref_fa, size_t ref_len, const char* tgt_fa, size_t tgt_len,
                 char** out, size_t* out_len) {
    orc_params p;
    orc_params_default(&p);
    return orc_compress_params(&p, ref_fa, ref_len, tgt_fa, tgt_len, out, out_len);
}

int orc_compress_params(const orc_params* prm, const char* ref_fa, size_t ref_len, const char* tgt_fa,
                        size_t tgt_len, char** out, size_t* out_len) {
    sb_t R = {0}, T = {0}, hdr = {0}, f = {0}, fin = {0};
    int has_header = 0, rc = ORC_OK;
    g_last_global = 0;
    g_last_switch = -1;
    ingest_reference(ref_fa, ref_len, &R);
    ingest_target(tgt_fa, tgt_len, &T, &hdr, &has_header);
    sb_reserve(&R, 1); sb_reserve(&T, 1);    /* non-NULL even when empty */

    if (has_header) { sb_put(&f, hdr.d, hdr.n); sb_putc(&f, '\n'); }     /* :337-339 */
    run_line(&f, T.d, (int64_t)T.n, 0);                                  /* :341-367 */
    sb_put(&f, "\n,\n", 3);                                              /* :368 */
    char* Ru = (char*)malloc(R.n + 1);
    char* Tu = (char*)malloc(T.n + 1);
    if (!Ru || !Tu) { rc = ORC_E_ALLOC; goto done; }
    for (size_t i = 0; i < R.n; i++) Ru[i] = c_toupper(R.d[i]);          /* :369-370 */
    for (size_t i = 0; i < T.n; i++) Tu[i] = c_toupper(T.d[i]);

    const int k = prm->k, k2 = prm->k2, L = prm->L, m = prm->m, T2 = prm->T2;   /* :373-379 */
    const float T1 = prm->T1;
    int64_t nRs = ((int64_t)R.n + L - 1) / L, nTs = ((int64_t)T.n + L - 1) / L;
    int64_t iters = nRs < nTs ? nRs : nTs;                              /* :392 */
    int mism = 0, local = prm->local != 0;
    if (!local) iters = 0;   /* local = 0: the global pass alone (parameter override, see header) */
    for (int64_t i = 0; i < iters && rc == ORC_OK; i++) {               /* :395 */
        const char* ri = Ru + i * L;
        int64_t nri = (int64_t)R.n - i * L; if (nri > L) nri = L;
        const char* ti = Tu + i * L;
        int64_t nti = (int64_t)T.n - i * L; if (nti > L) nti = L;
        int done_seg = 0;
        for (int pass = 0; pass < 2 && !done_seg; pass++) {
            orc_rec* recs; int64_t nrec;
            rc = orc_match(ri, nri, ti, nti, pass ? k2 : k, 0, 0, i * L, &recs, &nrec);
            if (rc != ORC_OK) break;
            if (any_match(recs, nrec)) {                               /* :402 / :429 */
                int64_t lit;
                rc = emit_records(&f, recs, nrec, ti, &lit);
                float ratio = (float)lit / (float)nti;                   /* :417 / :444 */
                if (ratio > T1 && has_non_n(ti, nti)) mism++;
                else mism = 0;
                done_seg = 1;
            }
            free(recs);
        }
        if (done_seg || rc != ORC_OK) continue;
        if (has_non_n(ti, nti)) mism++;                                 /* :454-460 */
        else mism = 0;
        if (mism > T2) { local = 0; g_last_switch = i; break; }         /* :462-473 */
    }
    if (rc != ORC_OK) goto done;
    if (local) {
        if (nTs > iters) sb_put(&f, Tu + iters * L, T.n - (size_t)(iters * L));   /* :476-481 */
    } else {
        /* global pass (:484-574): the file is rewritten from scratch */
        g_last_global = 1;
        f.n = 0;
        if (has_header) { sb_put(&f, hdr.d, hdr.n); sb_putc(&f, '\n'); }
        run_line(&f, T.d, (int64_t)T.n, 0);
        sb_putc(&f, '\n');
        run_line(&f, Tu, (int64_t)T.n, 1);                               /* :527-555 */
        sb_putc(&f, '\n');
        size_t nt2 = 0, nr2 = 0;                                         /* :556-557 */
        for (size_t i = 0; i < T.n; i++) if (Tu[i] != 'N') Tu[nt2++] = Tu[i];
        for (size_t i = 0; i < R.n; i++) if (Ru[i] != 'N') Ru[nr2++] = Ru[i];
        orc_rec* recs; int64_t nrec;
        rc = orc_match(Ru, (int64_t)nr2, Tu, (int64_t)nt2, k, m, 1, 0, &recs, &nrec);   /* :561 */
        if (rc == ORC_OK) rc = emit_records(&f, recs, nrec, Tu, NULL);   /* :564-573 */
        free(recs);
        if (rc != ORC_OK) goto done;
    }
    if (f.oom) { rc = ORC_E_ALLOC; goto done; }
    rc = delta_encode(f.d ? f.d : "", f.n, &fin);                       /* :579 */
    if (rc == ORC_E_DELTA_STOI) {
        /* the reference's file keeps the un-delta'd text (the throw happens before :296) */
        *out = f.d ? f.d : (char*)calloc(1, 1); *out_len = f.n; f.d = NULL;
        goto done;
    }
    if (rc == ORC_OK) {
        if (!fin.d) { fin.d = (char*)calloc(1, 1); }
        *out = fin.d; *out_len = fin.n; fin.d = NULL;
    }
done:
    free(Ru); free(Tu);
    free(R.d); free(T.d); free(hdr.d); free(f.d); free(fin.d);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* decompression -- decompression.cpp:21-114, 117-279, 316-323                                */
/* ------------------------------------------------------------------------------------------ */
/* std::getline on an ifstream: returns 0 (fail) when already at EOF. */
static int next_line(const char* s, size_t n, size_t* pos, const char** l, size_t* ln) {
    if (*pos >= n) return 0;
    const char* nl = memchr_from(s, n, *pos, '\n');
    size_t e = nl ? (size_t)(nl - s) : n;
    *l = s + *pos;
    *ln = e - *pos;
    *pos = nl ? e + 1 : n;
    return 1;
}

typedef struct { int* v; int64_t n, cap; int oom; } ivec_t;
static void iv_push(ivec_t* a, int x) {
    if (a->oom) return;
    if (a->n == a->cap) {
        int64_t nc = a->cap ? a->cap * 2 : 256;
        int* nv = (int*)realloc(a->v, (size_t)nc * sizeof(int));
        if (!nv) { a->oom = 1; return; }
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = x;
}
static int cmp_int(const void* a, const void* b) {
    int x = *(const int*)a, y = *(const int*)b;
    return (x > y) - (x < y);
}

/* decompression.cpp:126-163 (lowercase) and :166-206 (N): "(delta,len)" expands len
 * positions, a bare number expands one; each start is prev + delta.  Sorted afterwards. */
static int parse_positions(const char* s, size_t n, ivec_t* out) {
    int prev = 0;
    size_t pos = 0;
    while (pos < n) {
        if (s[pos] == '(') {
            const char* cp = memchr_from(s, n, pos, ')');
            if (!cp) return ORC_E_PARSE;        /* reference: substr to npos, undefined shape */
            size_t close = (size_t)(cp - s);
            const char* tok = s + pos + 1;
            size_t tn = close - pos - 1;
            const char* comma = (const char*)memchr(tok, ',', tn);
            if (!comma) return ORC_E_PARSE;
            int delta, len;
            if (stoi_like(tok, (size_t)(comma - tok), &delta)) return ORC_E_PARSE;
            if (stoi_like(comma + 1, (size_t)(tok + tn - comma - 1), &len)) return ORC_E_PARSE;
            int start = prev + delta;
            for (int j = 0; j < len; j++) iv_push(out, start + j);
            prev = start;
            pos = close + 1;
            if (pos < n && s[pos] == ',') pos++;
        } else {
            const char* cp = memchr_from(s, n, pos, ',');
            size_t e = cp ? (size_t)(cp - s) : n;
            if (e > pos) {
                int delta;
                if (stoi_like(s + pos, e - pos, &delta)) return ORC_E_PARSE;
                int start = prev + delta;
                iv_push(out, start);
                prev = start;
            }
            pos = cp ? e + 1 : n;
        }
    }
    if (out->oom) return ORC_E_ALLOC;
    if (out->n > 1) qsort(out->v, (size_t)out->n, sizeof(int), cmp_int);   /* (v may be NULL when empty) */
    return ORC_OK;
}

int orc_decompress(const char* rec, size_t rec_len, const char* ref_fa, size_t ref_len,
                   char** out, size_t* out_len) {
    int rc = ORC_OK;
    sb_t R = {0}, dec = {0}, res = {0}, fo = {0};
    ivec_t lp = {0}, np = {0};
    size_t pos = 0;
    const char *l1, *lower, *nline, *enc, *hdr = NULL;
    size_t n1, nlower, nnl, nenc, nhdr = 0;

    ingest_reference(ref_fa, ref_len, &R);                         /* :47-58 */
    sb_reserve(&R, 1);
    if (!next_line(rec, rec_len, &pos, &l1, &n1)) { rc = ORC_E_FORMAT; goto done; }   /* :68 */
    if (n1 > 0 && l1[0] == '>') {                                  /* :73-86 */
        hdr = l1; nhdr = n1;
        if (!next_line(rec, rec_len, &pos, &lower, &nlower) ||
            !next_line(rec, rec_len, &pos, &nline, &nnl) ||
            !next_line(rec, rec_len, &pos, &enc, &nenc)) { rc = ORC_E_FORMAT; goto done; }
    } else {                                                       /* :87-97 */
        lower = l1; nlower = n1;
        if (!next_line(rec, rec_len, &pos, &nline, &nnl) ||
            !next_line(rec, rec_len, &pos, &enc, &nenc)) { rc = ORC_E_FORMAT; goto done; }
    }
    if (!(nnl == 1 && nline[0] == ',')) {                          /* :105-109 erase 'N' */
        size_t w = 0;
        for (size_t i = 0; i < R.n; i++) if (R.d[i] != 'N') R.d[w++] = R.d[i];
        R.n = w;
    }
    for (size_t i = 0; i < R.n; i++) R.d[i] = c_toupper(R.d[i]);   /* :110 */

    if ((rc = parse_positions(lower, nlower, &lp)) != ORC_OK) goto done;    /* :126-164 */
    if ((rc = parse_positions(nline, nnl, &np)) != ORC_OK) goto done;       /* :166-207 */

    {                                                              /* :210-236 token decode */
        size_t i = 0;
        int prev_abs = 0;
        while (i < nenc) {
            if (enc[i] == '(') {
                const char* ep = memchr_from(enc, nenc, i, ')');
                const char* cp = memchr_from(enc, nenc, i, ',');
                if (!ep || !cp || cp > ep) { rc = ORC_E_PARSE; goto done; }
                int delta, length;
                if (stoi_like(enc + i + 1, (size_t)(cp - enc) - i - 1, &delta) ||
                    stoi_like(cp + 1, (size_t)(ep - cp) - 1, &length)) { rc = ORC_E_PARSE; goto done; }
                int abs_start = prev_abs + delta;
                prev_abs = abs_start;
                if ((long long)abs_start + length > (long long)R.n) { rc = ORC_E_RANGE; goto done; }
                if (abs_start < 0 || length < 0) { rc = ORC_E_PARSE; goto done; }
                sb_put(&dec, R.d + abs_start, (size_t)length);
                i = (size_t)(ep - enc) + 1;
            } else {
                sb_putc(&dec, enc[i]);
                i++;
            }
        }
    }
    {                                                              /* :241-252 insert N */
        int64_t total = (int64_t)dec.n + np.n, ti = 0, nj = 0;
        sb_reserve(&res, (size_t)total);
        for (int64_t i = 0; i < total; i++) {
            if (nj < np.n && np.v[nj] == i) { sb_putc(&res, 'N'); nj++; }
            else {
                if ((size_t)ti >= dec.n) { rc = ORC_E_PARSE; goto done; }   /* reference: UB */
                sb_putc(&res, dec.d[ti++]);
            }
        }
    }
    for (int64_t j = 0; j < lp.n; j++)                              /* :255-262 lowercase */
        if (lp.v[j] >= 0 && (size_t)lp.v[j] < res.n) res.d[lp.v[j]] = c_tolower(res.d[lp.v[j]]);
    /* :266-274 -- 50-column wrap, then a final "\n"; :322 header + "\n" in front */
    if (hdr) sb_put(&fo, hdr, nhdr);
    sb_putc(&fo, '\n');
    for (size_t p = 0; p < res.n; p += 50) {
        size_t c = res.n - p < 50 ? res.n - p : 50;
        sb_put(&fo, res.d + p, c);
        if (p + 50 < res.n) sb_putc(&fo, '\n');
    }
    sb_putc(&fo, '\n');
    if (fo.oom || res.oom || dec.oom) { rc = ORC_E_ALLOC; goto done; }
    *out = fo.d; *out_len = fo.n; fo.d = NULL;
done:
    free(R.d); free(dec.d); free(res.d); free(fo.d); free(lp.v); free(np.v);
    return rc;
}

void orc_free(void* p) { free(p); }
