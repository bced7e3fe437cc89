// local.hip -- local mode: per-segment match_sequences, the switch state machine, record text.
//
//   segment loop           compression.cpp:372-481
//   match_sequences(r_i, t_i, k, 0, false, i*L)   compression.cpp:36-179 with global=false
//   extend_alignment       compression.cpp:27-34
//
// One wavefront owns one 1000-base segment pair: both segments live in LDS (uppercased on load).
// The reference segment's k-mers are counting-sorted into 1024 hash buckets (one LDS atomic add
// per k-mer for its rank in the bucket, a wave scan for the bucket starts, one scatter) -- no
// probing, no CAS retries, and duplicate k-mers (poly-A, microsatellites) cost nothing extra.
// The target's "has any candidate" bits are computed lane-parallel from the buckets, and the walk
// is a wave-uniform loop that jumps from hit to hit.  A hit's candidates (its bucket's entries
// with the same k-mer) are extended by the whole wave one at a time, or one per lane when there
// are many, and reduced with the order-free form of the reference's selection loop (SURVEY.md
// A.4, tested against the oracle).  Segments are independent, so a launch covers every segment;
// the switch point is found afterwards by a state-machine scan.
#include "internal.h"

#include <cstdio>
#include <cstdlib>

namespace {

constexpr int WPB = 4;            // segments (waves) per block
constexpr int SEGB = 1024;        // LDS bytes per segment string (1000 + zero padding)
constexpr int NBB = 9;            // 512 k-mer buckets
constexpr int NB = 1 << NBB;
constexpr int MANY = 4;           // more candidates than this: extend one per lane
constexpr int32_t PASS_NEED_K2 = -3;   // a proved segment whose k pass found no match (launch_local_proven)

struct SegLds {
    uint8_t r[SEGB];
    uint8_t t[SEGB];
    uint32_t skey[1024];          // reference k-mer keys, grouped by bucket (first: the bucket counters)
    uint16_t spos[1024];          // their positions
    uint16_t bstart[NB + 1];      // bucket b holds entries [bstart[b], bstart[b+1])
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, int k) {
    for (int i = 0; i < k; i++) if (a[i] != b[i]) return false;
    return true;
}

// packed key (common.h) of the K-mer at s (LDS), scalar
template <int K>
__device__ __forceinline__ uint32_t seg_key(const uint8_t* s) {
    uint32_t code = 0;
#pragma unroll
    for (int i = 0; i < K; i++) {
        const uint32_t b = base2(s[i]);
        if (b > 3) return exotic_key(s, K);
        code |= b << (2 * i);
    }
    return code;
}

__device__ __forceinline__ uint64_t pick_key(int p, int pme) {
    const int d = p - pme;
    return ((uint64_t)(uint32_t)(d < 0 ? -d : d) << 32) | (uint32_t)p;
}

// uppercase 4 bytes (compression.cpp:369-370 toupper, C locale: only 'a'..'z' change), SWAR: a
// byte is lowercase iff its high bit is clear and (b & 0x7f) + 0x1f reaches 0x80 while + 0x05 does not
__device__ __forceinline__ uint32_t upper4(uint32_t w) {
    const uint32_t x = w & 0x7f7f7f7fu;
    const uint32_t lower = (x + 0x1f1f1f1fu) & ~(x + 0x05050505u) & ~w & 0x80808080u;
    return w ^ (lower >> 2);
}

// keys of the 16 K-mers starting at s[0..16) (s 16-byte aligned in LDS; 32 bytes readable)
template <int K>
__device__ __forceinline__ void keys16(const uint8_t* s, uint64_t& code, uint32_t& bad) {
    const uint32_t* w4 = reinterpret_cast<const uint32_t*>(s);
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = w4[i];
    pack_codes<8>(w, code, bad);
}

// extend_alignment (compression.cpp:27-34) of r[qc..] against t[y..] in LDS, whole wave, 4 bytes
// per lane per step; returns the extension clamped to [K, maxl]
template <int K>
__device__ __forceinline__ int wave_ext(const uint32_t* r4, const uint32_t* t4, int qc, int y, int maxl) {
    const int lane = lane_id();
    int l = maxl;
    for (int off = K; off < maxl; off += 256) {
        const int i = off + 4 * lane;
        int e = INT32_MAX;
        if (i < maxl) {
            const int ra = qc + i, ta = y + i;
            const uint32_t rv = __builtin_amdgcn_alignbyte(r4[(ra >> 2) + 1], r4[ra >> 2], (uint32_t)(ra & 3));
            const uint32_t tv = __builtin_amdgcn_alignbyte(t4[(ta >> 2) + 1], t4[ta >> 2], (uint32_t)(ta & 3));
            const uint32_t x = rv ^ tv;
            if (x) e = i + (__builtin_ctz(x) >> 3);
            else if (maxl - i <= 4) e = maxl;
        }
        const unsigned long long sm = __ballot(e != INT32_MAX);
        if (sm) { l = lane_val(e, first_lane(sm)); break; }
    }
    if (l > maxl) l = maxl;
    if (l < K) l = K;
    return l;
}

// SCCG_DEBUG: phase ticks (10 ns) summed over segments: load, keys, insert, hits, walk, count
__device__ unsigned long long g_local_dbg[16];

// One segment with one k (pass 1: k = 14, pass 2: k2 = 10 on a segment pass 1 left without a match,
// keeping pass 1's non-N flag); returns its statistics (wave-uniform), the records are in recs.
// The words of a segment pair one lane loads (dword i = lane + 64 j, j < 4): the persistent local
// pass loads its next segment's words before working on the current one, so the HBM round trip of
// the load overlaps a whole segment's LDS work instead of starting each segment.
struct SegWords {
    uint32_t r[SEGB / 256], t[SEGB / 256];
};
__device__ __forceinline__ void seg_words_load(SegWords& W, int64_t seg, const uint8_t* __restrict__ R, int64_t nR,
                                               const uint8_t* __restrict__ T, int64_t nT) {
    const int lane = lane_id();
    const int64_t base = seg * SEG_L;
    const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L);
    const int nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);
    const uint32_t* R4 = reinterpret_cast<const uint32_t*>(R + base);
    const uint32_t* T4 = reinterpret_cast<const uint32_t*>(T + base);
#pragma unroll
    for (int j = 0; j < SEGB / 256; j++) {
        const int i = lane + 64 * j, b0 = 4 * i;
        W.r[j] = b0 < nr ? R4[i] : 0u;
        W.t[j] = b0 < nt ? T4[i] : 0u;
    }
}

// Both segments into LDS, uppercased (compression.cpp:369-370, :386-389); base is a multiple of 1000,
// so the dword loads are aligned; bytes past a segment end read as 0.  Returns "the target segment
// holds a byte other than 'N'" (compression.cpp:419), wave-uniform.
__device__ __forceinline__ bool seg_load(SegLds& L, int64_t seg, int upper, const uint8_t* __restrict__ R, int64_t nR,
                                         const uint8_t* __restrict__ T, int64_t nT, const SegWords* pre) {
    const int lane = lane_id();
    const int64_t base = seg * SEG_L;
    const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L);
    const int nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);
    bool non_n = false;
    const uint32_t* R4 = reinterpret_cast<const uint32_t*>(R + base);
    const uint32_t* T4 = reinterpret_cast<const uint32_t*>(T + base);
    uint32_t* r4 = reinterpret_cast<uint32_t*>(L.r);
    uint32_t* t4 = reinterpret_cast<uint32_t*>(L.t);
#pragma unroll
    for (int j = 0; j < SEGB / 256; j++) {
        const int i = lane + 64 * j, b0 = 4 * i;
        uint32_t rw, tw;
        if (pre) { rw = pre->r[j]; tw = pre->t[j]; }
        else { rw = b0 < nr ? R4[i] : 0u; tw = b0 < nt ? T4[i] : 0u; }
        if (nr - b0 < 4) rw &= nr - b0 <= 0 ? 0u : (1u << (8 * (nr - b0))) - 1u;
        if (nt - b0 < 4) tw &= nt - b0 <= 0 ? 0u : (1u << (8 * (nt - b0))) - 1u;
        if (upper) { rw = upper4(rw); tw = upper4(tw); }
        r4[i] = rw;
        t4[i] = tw;
#pragma unroll
        for (int q = 0; q < 4; q++) non_n |= (b0 + q < nt && (uint8_t)(tw >> (8 * q)) != 'N');
    }
    non_n = __ballot(non_n) != 0;
    wave_sync();
    return non_n;
}

// Class-0 proof of a segment pair in LDS (the switch scan's common case, compression.cpp:400-416):
// the k = 14 pass succeeds with at most half of the target literal, without hashing or walking.  A
// target position whose k-mer occurs in the reference segment has a candidate, so the walk never
// visits it as a literal step (literal bases are positions without a candidate, plus at most the
// K - 1 after the last k-mer start); and one such position makes the pass find a match.  Positions
// "with a candidate" are shown on a few diagonals d: T[i..i+K) == R[i+d..i+d+K).  The diagonals
// come from 8 sampled target k-mers looked up among the reference segment's k-mer keys.  A segment
// the proof cannot settle takes the walk as before; the proof only ever answers "class 0".
constexpr int PROOF_SAMPLES = 8, PROOF_DIAGS = 4;
__device__ __forceinline__ bool seg_prove(const uint8_t* Lr, const uint8_t* Lt, int nr, int nt) {
    constexpr int K = 14;
    constexpr uint32_t MASK = (1u << (2 * K)) - 1u, KM = (1u << K) - 1u;
    const int lane = lane_id();
    const int lastr = nr - K, lastk = nt - K;
    if (lastr < 0 || lastk < 0) return false;
    // reference keys of positions 16 lane .. 16 lane + 15 (invalid: 0xffffffff)
    uint32_t rk[16];
    {
        const int p0 = 16 * lane;
        uint64_t code = 0;
        uint32_t bad = ~0u;
        if (p0 <= lastr) keys16<K>(&Lr[p0], code, bad);
#pragma unroll
        for (int st = 0; st < 16; st++)
            rk[st] = (p0 + st <= lastr && !((bad >> st) & KM)) ? (uint32_t)(code >> (2 * st)) & MASK : 0xffffffffu;
    }
    // sampled target k-mers: lane j < PROOF_SAMPLES holds the key at y_j = j * lastk / PROOF_SAMPLES
    uint32_t tk = 0xfffffffeu;
    const int yl = lane < PROOF_SAMPLES ? (int)((int64_t)lane * lastk / PROOF_SAMPLES) : 0;
    if (lane < PROOF_SAMPLES) {
        uint32_t w[4], bad;
        uint64_t code;
        loadw<4>(&Lt[yl], w);
        pack_codes<4>(w, code, bad);
        if (!(bad & KM)) tk = (uint32_t)code & MASK;
    }
    int32_t dg[PROOF_DIAGS];
    int nd = 0;
    for (int j = 0; j < PROOF_SAMPLES && nd < PROOF_DIAGS; j++) {
        const uint32_t kj = lane_val(tk, j);
        if (kj == 0xfffffffeu) continue;
        uint32_t m = 0;
#pragma unroll
        for (int st = 0; st < 16; st++) m |= (uint32_t)(rk[st] == kj) << st;
        const unsigned long long b = __ballot(m != 0);
        if (!b) continue;
        const int fl = first_lane(b);
        const int32_t d = 16 * fl + __builtin_ctz(lane_val(m, fl)) - lane_val(yl, j);
        bool dup = false;
        for (int q = 0; q < nd; q++) dup |= dg[q] == d;
        if (!dup) dg[nd++] = d;
    }
    if (!nd) return false;
    // positions 16 lane .. +15 covered on some diagonal: 14 equal bytes from i (and from i + d)
    const int i0 = 16 * lane;
    uint32_t tw[8];
    {
        const uint32_t* t4 = reinterpret_cast<const uint32_t*>(Lt) + 4 * lane;
#pragma unroll
        for (int q = 0; q < 8; q++) tw[q] = lane < 63 || q < 4 ? t4[q] : 0u;
    }
    uint32_t cov = 0;
    for (int q = 0; q < nd; q++) {
        const int32_t d = dg[q];
        int ra = i0 + d;   // R bytes ra .. ra + 31 (a lane whose stretch leaves the buffer proves nothing)
        const bool inside = ra >= 0 && ra <= SEGB - 36;
        ra = inside ? ra : 0;
        uint32_t rw[8];
        loadw<8>(&Lr[ra], rw);
        uint32_t e = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) e |= ((~nz_bytes(tw[w] ^ rw[w])) & 0xfu) << (4 * w);
        uint32_t c = e & (e >> 1);
        c &= c >> 2;
        c &= c >> 4;
        c &= c >> 6;   // bit i: bytes i .. i + 13 equal
        // valid starts: i <= lastk, 0 <= i + d <= lastr, and the R bytes read really were R[i + d ...]
        uint32_t v = 0xffffu;
        const int tv = lastk - i0 + 1;                 // i0 + st <= lastk
        v &= tv <= 0 ? 0u : (tv >= 16 ? 0xffffu : (1u << tv) - 1u);
        const int rv = lastr - (i0 + d) + 1;           // i0 + d + st <= lastr
        v &= rv <= 0 ? 0u : (rv >= 16 ? 0xffffu : (1u << rv) - 1u);
        if (!inside) v = 0;
        cov |= c & v;
    }
    const int tv = lastk - i0 + 1;
    const uint32_t tvm = tv <= 0 ? 0u : (tv >= 16 ? 0xffffu : (1u << tv) - 1u);
    const int unc = wave_sum((int)__popc(tvm & ~cov));
    const bool any = __ballot(cov != 0) != 0;
    return any && 2 * (unc + (nt - 1 - lastk)) <= nt;
}

// H of compression.cpp:41-47 for one segment: every K-mer of the reference segment in LDS,
// counting-sorted by bucket (lane l owns starts 16l..16l+15); L.bstart[b] .. L.bstart[b+1] hold
// bucket b's keys (L.skey) and positions (L.spos).
template <int K>
__device__ __forceinline__ void seg_table(SegLds& L, int nr) {
    const int lane = lane_id();
    constexpr uint32_t MASK = (1u << (2 * K)) - 1u, KM = (1u << K) - 1u;
    const int lastr = nr - K;
    uint32_t* cnt = L.skey;   // bucket counters live where the keys go later
    for (int i = lane; i < NB; i += 64) cnt[i] = 0;
    wave_sync();
    {
        const int p0 = lane * 16;
        uint64_t code = 0;
        uint32_t bad = 0;
        if (p0 <= lastr) keys16<K>(&L.r[p0], code, bad);   // lanes past lastr own no k-mer
        uint32_t key[16], rank[16];
#pragma unroll
        for (int st = 0; st < 16; st++) {
            const int p = p0 + st;
            key[st] = 0;
            if (p <= lastr) {
                key[st] = (bad >> st) & KM ? exotic_key(&L.r[p], K) : (uint32_t)(code >> (2 * st)) & MASK;
                rank[st] = atomicAdd(&cnt[slot_hash(key[st], NBB)], 1u);
            }
        }
        wave_sync();
        // bucket starts: exclusive scan of the counts (NB / 64 buckets per lane)
        constexpr int BPL = NB / 64;
        uint32_t c[BPL], run = 0;
#pragma unroll
        for (int i = 0; i < BPL; i++) { c[i] = cnt[BPL * lane + i]; run += c[i]; }
        const uint32_t incl = wave_incl_add(run);
        uint32_t o = incl - run;
#pragma unroll
        for (int i = 0; i < BPL; i++) { L.bstart[BPL * lane + i] = (uint16_t)o; o += c[i]; }
        if (lane == 63) L.bstart[NB] = (uint16_t)o;
        wave_sync();
#pragma unroll
        for (int st = 0; st < 16; st++) {
            const int p = p0 + st;
            if (p <= lastr) {
                const uint32_t at = L.bstart[slot_hash(key[st], NBB)] + rank[st];
                L.skey[at] = key[st];
                L.spos[at] = (uint16_t)p;
            }
        }
    }
    wave_sync();
}

// Hit positions of the target segment: y in [0, nt - K] whose K-mer occurs among the reference
// segment's (compression.cpp:77 H.find succeeds); the table is seg_table<K>'s.  Pure keys only
// (the caller has excluded segments holding bytes outside ACGT).  Counts up to at least `cap`.
template <int K>
__device__ __forceinline__ int seg_hits(const SegLds& L, int nr, int nt) {
    const int lane = lane_id();
    constexpr uint32_t MASK = (1u << (2 * K)) - 1u;
    const int lastk = nt - K;
    if (nr < K || lastk < 0) return 0;
    const int p0 = lane * 16;
    uint64_t code = 0;
    uint32_t bad = 0;
    if (p0 <= lastk) keys16<K>(&L.t[p0], code, bad);
    int h = 0;
#pragma unroll
    for (int st = 0; st < 16; st++) {
        if (p0 + st <= lastk) {
            const uint32_t key = (uint32_t)(code >> (2 * st)) & MASK;
            const uint32_t b = slot_hash(key, NBB);
            const int e1 = (int)L.bstart[b + 1];
            bool hit = false;
            for (int e = (int)L.bstart[b]; e < e1 && !hit; e++) hit = L.skey[e] == key;
            h += hit;
        }
    }
    return wave_sum(h);
}

template <int K, bool DBG>
__device__ __forceinline__ SegStat local_segment(SegLds& L, int64_t seg, int pass, int non_n_prev, int upper,
                                                 const uint8_t* __restrict__ R, int64_t nR, const uint8_t* __restrict__ T,
                                                 int64_t nT, uint32_t* __restrict__ recs, const SegWords* pre = nullptr,
                                                 int loaded = -1) {
    const int lane = lane_id();
    const int64_t base = seg * SEG_L;
    const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L);
    const int nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);
    constexpr uint32_t MASK = (1u << (2 * K)) - 1u, KM = (1u << K) - 1u;
    uint64_t tq = DBG ? wall_clock64() : 0, tph[5] = {0, 0, 0, 0, 0};
    auto tick = [&](int i) {
        if (DBG) { const uint64_t t = wall_clock64(); tph[i] += t - tq; tq = t; }
    };

    // ---- both segments in LDS (loaded >= 0: already there, `loaded` = its non-N flag)
    const bool non_n = loaded >= 0 ? loaded != 0 : seg_load(L, seg, upper, R, nR, T, nT, pre);
    tick(0);

    seg_table<K>(L, nr);
    const int lastr = nr - K;
    wave_sync();
    tick(1);
    tick(2);
    tick(3);

    // ---- the greedy walk (compression.cpp:64-161), wave-uniform.  The next target position with
    //      a candidate (compression.cpp:77 "H.find") is found 64 positions at a time from idx: an
    //      aligned segment takes a step or two, so probing only where the walk goes is far cheaper
    //      than a hit bit for every target k-mer.
    const int lastk = nt - K;
    uint32_t* out = recs + seg * SEG_REC_CAP;
    int idx = 0, pme = -1, nrec = 0, nmatch = 0, lit = 0, firstp = -1, lastp = -1;
    for (;;) {
        // next target position >= idx with a candidate (and its key)
        int nxt = -1;
        uint32_t key = 0;
        if (lastr >= 0) {
            for (int p0 = idx; p0 <= lastk; p0 += 64) {
                const int p = p0 + lane;
                bool hit = false;
                uint32_t pkey = 0;
                if (p <= lastk) {
                    uint32_t w[4], bad;
                    uint64_t code;
                    loadw<4>(&L.t[p], w);
                    pack_codes<4>(w, code, bad);
                    pkey = bad & KM ? exotic_key(&L.t[p], K) : (uint32_t)code & MASK;
                    const uint32_t key = pkey;
                    const uint32_t b = slot_hash(key, NBB);
                    const int e1 = (int)L.bstart[b + 1];
                    for (int e = (int)L.bstart[b]; e < e1; e++) {
                        if (L.skey[e] == key && (key < KEY_EXOTIC || bytes_eq(&L.r[L.spos[e]], &L.t[p], K))) {
                            hit = true;
                            break;
                        }
                    }
                }
                const unsigned long long hm = __ballot(hit);
                if (hm) { nxt = p0 + first_lane(hm); key = lane_val(pkey, first_lane(hm)); break; }
            }
        }
        if (nxt < 0) break;
        if (nxt > idx) {
            if (lane == 0) out[nrec] = ((uint32_t)idx << 11) | (uint32_t)(nxt - idx);
            nrec++;
            lit += nxt - idx;
        }
        const uint32_t bk = slot_hash(key, NBB);
        const int e0 = (int)L.bstart[bk], e1 = (int)L.bstart[bk + 1];
        const uint32_t* r4 = reinterpret_cast<const uint32_t*>(L.r);
        const uint32_t* t4 = reinterpret_cast<const uint32_t*>(L.t);
        // candidates: the bucket's entries holding this k-mer, 64 entries per step
        int bl = 0, bcnt = 0;
        bool bhas0 = false;
        uint64_t bkey = ~0ull;
        // A candidate's extension is bounded by min(nr - q, nt - nxt); one whose bound is below the
        // best extension found cannot change the pick.  With more than one batch of entries, the
        // candidate with the largest bound (the least q) is extended first, so the bound prunes the
        // rest (all-N / homopolymer segments: ~1000 candidates, one of which reaches the end).
        int lb = 0;
        if (e1 - e0 > 64) {
            int qmin = INT32_MAX;
            for (int eb = e0; eb < e1; eb += 64) {
                const int e = eb + lane;
                if (e < e1 && L.skey[e] == key) {
                    const int q = L.spos[e];
                    if (q < qmin && (key < KEY_EXOTIC || bytes_eq(&L.r[q], &L.t[nxt], K))) qmin = q;
                }
            }
            qmin = wave_min(qmin);
            if (qmin != INT32_MAX)
                lb = wave_ext<K>(r4, t4, qmin, nxt, (nr - qmin) < (nt - nxt) ? (nr - qmin) : (nt - nxt));
        }
        for (int eb = e0; eb < e1; eb += 64) {
            const int e = eb + lane;
            int q = -1;
            if (e < e1 && L.skey[e] == key) {
                q = L.spos[e];
                if (key >= KEY_EXOTIC && !bytes_eq(&L.r[q], &L.t[nxt], K)) q = -1;
            }
            const int thr = bl > lb ? bl : lb;
            if (q >= 0 && ((nr - q) < (nt - nxt) ? (nr - q) : (nt - nxt)) < thr) q = -1;   // pruned (see above)
            unsigned long long cm = __ballot(q >= 0);
            if (__popcll(cm) <= MANY) {
                while (cm) {   // few candidates: the whole wave extends each
                    const int cl = __ffsll((long long)cm) - 1;
                    cm &= cm - 1;
                    const int qc = lane_val(q, cl);
                    const int maxl = (nr - qc) < (nt - nxt) ? (nr - qc) : (nt - nxt);
                    if (maxl < bl) continue;   // cannot reach the best extension: no effect on the pick
                    const int l = wave_ext<K>(r4, t4, qc, nxt, maxl);
                    if (l > bl) { bl = l; bcnt = 1; bhas0 = (qc == 0); bkey = qc ? pick_key(qc, pme) : ~0ull; }
                    else if (l == bl) {
                        bcnt++;
                        if (qc == 0) bhas0 = true;
                        else { const uint64_t pk = pick_key(qc, pme); bkey = pk < bkey ? pk : bkey; }
                    }
                }
            } else {   // many candidates (repeats): one per lane, 4 bytes per step
                int l = 0;
                if (q >= 0) {
                    const int maxl = (nr - q) < (nt - nxt) ? (nr - q) : (nt - nxt);
                    l = K;
                    while (l < maxl) {   // 16 bytes per step
                        uint32_t rv[4], tv[4];
                        loadw<4>(&L.r[q + l], rv);
                        loadw<4>(&L.t[nxt + l], tv);
                        int d = 16;
#pragma unroll
                        for (int w = 3; w >= 0; w--) {
                            const uint32_t x = rv[w] ^ tv[w];
                            if (x) d = 4 * w + (__builtin_ctz(x) >> 3);
                        }
                        l += d;
                        if (d < 16) break;
                    }
                    if (l > maxl) l = maxl;
                }
                const int lm = wave_max(l);
                const int cnt = (int)__popcll(__ballot(q >= 0 && l == lm));
                const bool h0 = __ballot(q == 0 && l == lm) != 0;
                const uint64_t mk = wave_min((q > 0 && l == lm) ? pick_key(q, pme) : ~0ull);
                if (lm > bl) { bl = lm; bcnt = cnt; bhas0 = h0; bkey = mk; }
                else if (lm == bl) { bcnt += cnt; bhas0 |= h0; bkey = mk < bkey ? mk : bkey; }
            }
        }
        const int Lm = bl;
        uint64_t pk;
        if (bcnt >= 2 && bhas0) pk = bkey;                 // pn==0 sentinel (compression.cpp:118, :125)
        else {
            const uint64_t k0 = bhas0 ? pick_key(0, pme) : ~0ull;
            pk = k0 < bkey ? k0 : bkey;
        }
        const int p = (int)(uint32_t)pk;
        if (lane == 0) out[nrec] = 0x80000000u | ((uint32_t)p << 11) | (uint32_t)Lm;
        nrec++;
        nmatch++;
        if (firstp < 0) firstp = p;
        lastp = p;
        pme = p + Lm - 1;                              // compression.cpp:149
        idx = nxt + Lm;                                // compression.cpp:159
    }
    if (idx < nt) {                                    // compression.cpp:164-167
        if (lane == 0) out[nrec] = ((uint32_t)idx << 11) | (uint32_t)(nt - idx);
        nrec++;
        lit += nt - idx;
    }
    if (DBG) {
        tick(4);
        if (lane == 0) {
            for (int i = 0; i < 5; i++) atomicAdd(&g_local_dbg[i], (unsigned long long)tph[i]);
            atomicAdd(&g_local_dbg[5], 1ull);
            const unsigned long long tot = tph[0] + tph[1] + tph[2] + tph[3] + tph[4];
            if (tot > atomicMax(&g_local_dbg[6], tot)) {   // racy snapshot of the slowest segment (diagnostics)
                for (int i = 0; i < 5; i++) g_local_dbg[8 + i] = tph[i];
                g_local_dbg[13] = (unsigned long long)seg;
                g_local_dbg[14] = (unsigned long long)nmatch;
            }
        }
    }
    SegStat s;
    s.nrec = nrec;
    s.nmatch = nmatch;
    s.lit = lit;
    s.pass = nmatch ? pass : 0;
    s.non_n = pass == 1 ? (int)non_n : non_n_prev;
    s.first_p = firstp;
    s.last_p = lastp;
    s.pad = nt;
    return s;
}

// Segments [seg0, seg_end) with one k, a wave per segment (grid-stride).
template <int K, bool DBG>
__global__ __launch_bounds__(SCCG_BLOCK) void k_local_pass(int pass, int upper, const uint8_t* __restrict__ R, int64_t nR,
                                                           const uint8_t* __restrict__ T, int64_t nT, int64_t seg0,
                                                           int64_t seg_end, uint32_t* __restrict__ recs,
                                                           SegStat* __restrict__ stat) {
    __shared__ SegLds lds_all[WPB];
    const int w = wave_in_block();
    const int64_t G = (int64_t)gridDim.x * WPB;
    for (int64_t seg = seg0 + (int64_t)blockIdx.x * WPB + w; seg < seg_end; seg += G) {
        if (pass == 2 && stat[seg].pass != 0) continue;
        if (pass == 3 && stat[seg].pass != PASS_PROVEN) continue;   // (a proof means the k pass succeeds)
        if (pass == 4 && stat[seg].pass != PASS_NEED_K2) continue;
        SegStat st = local_segment<K, DBG>(lds_all[w], seg, pass == 3 ? 1 : pass == 4 ? 2 : pass,
                                           pass == 2 || pass == 4 ? stat[seg].non_n : 0, upper, R, nR, T, nT, recs);
        if (pass == 3 && st.pass == 0) st.pass = PASS_NEED_K2;   // (never, if the proof holds)
        if (lane_id() == 0) stat[seg] = st;
        wave_sync();   // the next segment reuses this wave's LDS
    }
}

// ---------------------------------------------------------------------------------------------
// All local segments in one launch (compress).  The grid is the resident capacity and wave i takes
// segments i, i + G, ... (so the front of processed segments advances in order); each runs k = 14
// and, without a match, k2 = 10 (compression.cpp:372-474).
// The switch state machine (compression.cpp:462-473) is a window predicate: its counter before
// segment e is the number of consecutive class-1/2 segments just before e (class 0/3 resets it),
// so the switch happens at the first e of class 2 whose 4 predecessors are all class 1 or 2.
// A wave publishes its segment's class (tagged with the call's generation, so the array is never
// cleared) and checks the 5 windows holding it; a complete window with that shape lowers ctl[1],
// and segments past ctl[1] are never started: their work would be discarded.  The class traffic is
// relaxed agent-scope atomics (no cache maintenance; a window two waves complete at once may go
// unseen, which only delays the exit): k_switch_final recomputes the first switch from the
// published classes after the launch (all segments up to it were computed).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int seg_class(const SegStat& s) {
    // 0 good, 1 success-but-bad (mism++ without check), 2 failed non-N (mism++ + check), 3 failed all-N
    if (s.pass) return (2 * s.lit > s.pad && s.non_n) ? 1 : 0;   // (float)lit/len > 0.5f
    return s.non_n ? 2 : 3;
}
__device__ __forceinline__ bool mism(int c) { return c == 1 || c == 2; }

// The lengths come from device memory (the FASTA strips' counts), so the launch needs no host sync.
__device__ __forceinline__ int32_t seg_count(int64_t nR, int64_t nT) {
    const int64_t a = (nR + SEG_L - 1) / SEG_L, b = (nT + SEG_L - 1) / SEG_L;
    const int64_t n = a < b ? a : b;
    return n >= INT32_MAX / 2 ? 0 : (int32_t)n;   // beyond int positions: the host reports it
}

#ifndef LOCAL_WAVES_PER_EU
#define LOCAL_WAVES_PER_EU 4   // the LDS allows 4 waves/SIMD (4 blocks of SegLds x 4); VGPRs must fit 128
#endif
// prove: each segment is first tried by the class-0 proof (seg_prove); a proved segment publishes
// class 0 without its records (PASS_PROVEN: a pair that stays local computes them afterwards,
// launch_local_proven) -- only the switch scan of a pair that goes global skips its walk.
template <bool DBG>
__global__ __launch_bounds__(SCCG_BLOCK) __attribute__((amdgpu_waves_per_eu(LOCAL_WAVES_PER_EU))) void k_local_all(const uint8_t* __restrict__ R, const int64_t* __restrict__ dnR,
                                                          const uint8_t* __restrict__ T, const int64_t* __restrict__ dnT,
                                                          uint32_t* __restrict__ recs, SegStat* __restrict__ stat,
                                                          int32_t* __restrict__ cls, int32_t gen, int32_t* __restrict__ ctl,
                                                          int prove) {
    __shared__ SegLds lds_all[WPB];
    const int64_t nR = *dnR, nT = *dnT;
    const int32_t nseg = seg_count(nR, nT);
    const int w = wave_in_block(), lane = lane_id();
    SegLds& L = lds_all[w];
    const int32_t G = (int32_t)gridDim.x * WPB;
    SegWords cur, nxt;
    int32_t seg = (int32_t)blockIdx.x * WPB + w;
    // (a probe window already decided the mode: ctl[1] = -1, nothing to start)
    if (uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 0) return;
    if (seg < nseg) seg_words_load(cur, seg, R, nR, T, nT);
    for (; seg < nseg; seg += G) {
        if (seg > uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) break;
        if (seg + G < nseg) seg_words_load(nxt, seg + G, R, nR, T, nT);   // in flight during this segment
        const bool non_n = seg_load(L, seg, 1, R, nR, T, nT, &cur);
        SegStat st;
        int c;
        const int64_t base = (int64_t)seg * SEG_L;
        const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L), nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);
        if (prove && seg_prove(L.r, L.t, nr, nt)) {
            // class 0 without its records: a pair that stays local computes them later (PASS_PROVEN)
            st = SegStat{0, 0, 0, PASS_PROVEN, (int)non_n, -1, -1, nt};
            c = 0;
            if (DBG && lane == 0) atomicAdd(&g_local_dbg[15], 1ull);
        } else {
            // (unproved: re-read the bound before the k pass as well -- a switch found during the proof)
            if (seg > uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) break;
            st = local_segment<14, DBG>(L, seg, 1, 0, 1, R, nR, T, nT, recs, nullptr, (int)non_n);
            if (!st.pass) {
                // a switch found meanwhile at or before this segment: its class is never read (no
                // window past the first switch counts), so the k2 pass is skipped and nothing published
                if (seg > uni(__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) break;
                wave_sync();
                // (the segment strings are still in LDS: the k pass only reads them)
                st = local_segment<10, DBG>(L, seg, 2, st.non_n, 1, R, nR, T, nT, recs, nullptr, 1);
            }
            c = seg_class(st);
        }
        if (lane == 0) stat[seg] = st;
        if (lane == 0) __hip_atomic_store(&cls[seg], (gen << 2) | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // classes of seg-4 .. seg+4 (lane i holds seg-4+i; -1 = not published in this call)
        const int32_t idx = seg - 4 + lane;
        int v = -1;
        if (lane < 9 && lane != 4 && idx >= 0 && idx < nseg) {
            const int32_t t = __hip_atomic_load(&cls[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = (t >> 2) == gen ? (t & 3) : -1;
        }
        if (lane == 4) v = c;
        int k[9];
#pragma unroll
        for (int i = 0; i < 9; i++) k[i] = lane_val(v, i);
        int32_t hit = INT32_MAX;
#pragma unroll
        for (int m = 8; m >= 4; m--)   // window ending at seg - 4 + m
            if (k[m] == 2 && mism(k[m - 1]) && mism(k[m - 2]) && mism(k[m - 3]) && mism(k[m - 4]) && seg - 4 + m >= 4)
                hit = seg - 4 + m;
        if (hit != INT32_MAX && lane == 0)
            __hip_atomic_fetch_min(&ctl[1], hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();   // the next segment reuses this wave's LDS
        cur = nxt;
    }
}

// ---------------------------------------------------------------------------------------------
// Switch probe (round 6; the default unless the caller asks for the exact switch segment,
// SCCG_OPT_EXACT_SWITCH).  The machine switches iff SOME window of 5 class-1/2 segments ends in a
// class-2 segment (the counter is a run length reset by class 0/3, and a window at e makes it switch
// at e unless it did before), and a switching pair's record file does not depend on where it
// switched (compression.cpp:462-473 -- the file is truncated and the global pass regenerates it,
// :484-574).  So one complete window anywhere decides the mode.  Drifted hg/T2T pairs are full of
// them past their first switch (segment pairs that no longer overlap fail both passes or match by
// chance: classes 1 and 2), so PROBE_RUNS runs of PROBE_RUN consecutive segments spread over the pair
// are classified first, one wave per segment, from their k2 hit counts alone (below).  The host reads
// the 128 classes back behind the walk's first rounds (sccg_api.cpp decide_probe): a window among
// them decides the pair global and the in-order pass (k_local_all) is never launched; otherwise it
// runs as before.
// ---------------------------------------------------------------------------------------------
constexpr int PROBE_RUN = 8, PROBE_RUNS = SCCG_PROBE_RUNS, PROBE_MIN_SEGS = 512;
static_assert(PROBE_RUN * PROBE_RUNS == PROBE_PAIRS, "internal.h's probe size");
// run r starts at (r + 1) nseg / (RUNS + 1): spread over the pair, clear of its last segments
// (telomere gaps)
__device__ __forceinline__ int32_t probe_run_start(int32_t r, int32_t nseg) {
    return (int32_t)((int64_t)(r + 1) * nseg / (PROBE_RUNS + 1)) - PROBE_RUN / 2;
}
// bytes of w (the first `valid` of its 4) outside A, C, G, T (uppercased)
__device__ __forceinline__ bool non_acgt4(uint32_t w, int valid) {
    bool bad = false;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t b = (w >> (8 * q)) & 0xffu;
        bad |= q < valid && b != 'A' && b != 'C' && b != 'G' && b != 'T';
    }
    return bad;
}
// SCCG_DEBUG: per probed segment {start, after the load, -, -, end} (wall clock), its class and k2 hits
__device__ unsigned long long g_probe_dbg[PROBE_RUNS * PROBE_RUN][6];
// One wave per workgroup: beside the other pairs' walks and strips, which fill most CUs' registers,
// a 9 KiB / one-wave group finds a slot at once (an 8-wave group of a whole run, 74 KiB of LDS and
// two waves' registers on every SIMD, waited ~0.5 ms for a CU to drain).  Each wave writes its
// segment's class (or -1) and index to pout; the host looks for windows (local_probe_window).
// The probed segments (slot i = run i / RUN, segment i % RUN of it; -1: none), for the gathers of
// their stripped bytes (ingest.hip k_strip_gather) and the probe.
__global__ void k_probe_segs(const int64_t* __restrict__ dnR, const int64_t* __restrict__ dnT, int32_t* __restrict__ segs) {
    const int32_t nseg = seg_count(*dnR, *dnT);
    for (int i = (int)threadIdx.x; i < PROBE_RUNS * PROBE_RUN; i += (int)blockDim.x)
        segs[i] = nseg < PROBE_MIN_SEGS ? -1 : probe_run_start(i / PROBE_RUN, nseg) + i % PROBE_RUN;
}

// Both segments of slot i from the gathered copies (SEG_GATHER_B bytes per slot; bytes past a
// segment's end read as 0), uppercased as seg_load does.
__device__ __forceinline__ void seg_load_gathered(SegLds& L, int slot, int nr, int nt, const uint8_t* __restrict__ gR,
                                                  const uint8_t* __restrict__ gT) {
    const int lane = lane_id();
    const uint32_t* R4 = reinterpret_cast<const uint32_t*>(gR + (size_t)slot * SEG_GATHER_B);
    const uint32_t* T4 = reinterpret_cast<const uint32_t*>(gT + (size_t)slot * SEG_GATHER_B);
    uint32_t* r4 = reinterpret_cast<uint32_t*>(L.r);
    uint32_t* t4 = reinterpret_cast<uint32_t*>(L.t);
#pragma unroll
    for (int j = 0; j < SEGB / 256; j++) {
        const int i = lane + 64 * j, b0 = 4 * i;
        uint32_t rw = b0 < nr ? R4[i] : 0u, tw = b0 < nt ? T4[i] : 0u;
        if (nr - b0 < 4) rw &= nr - b0 <= 0 ? 0u : (1u << (8 * (nr - b0))) - 1u;
        if (nt - b0 < 4) tw &= nt - b0 <= 0 ? 0u : (1u << (8 * (nt - b0))) - 1u;
        r4[i] = upper4(rw);
        t4[i] = upper4(tw);
    }
    wave_sync();
}

template <bool DBG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LOCAL_WAVES_PER_EU))) void k_local_probe(
    const uint8_t* __restrict__ gR, const int64_t* __restrict__ dnR, const uint8_t* __restrict__ gT,
    const int64_t* __restrict__ dnT, const int32_t* __restrict__ segs, int32_t* __restrict__ pout) {
    unsigned long long tk[5] = {DBG ? (unsigned long long)wall_clock64() : 0ull, 0, 0, 0, 0};
    __shared__ SegLds L;
    const int64_t nR = *dnR, nT = *dnT;
    const int32_t nseg = seg_count(nR, nT);
    const int lane = lane_id();
    if (nseg < PROBE_MIN_SEGS) {   // (uniform) small pairs: the in-order pass is cheap
        if (lane == 0) { pout[blockIdx.x] = -1; pout[PROBE_RUNS * PROBE_RUN + blockIdx.x] = -1; }
        return;
    }
    const int32_t seg = segs[blockIdx.x];
    const int64_t base = (int64_t)seg * SEG_L;
    const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L), nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);
    seg_load_gathered(L, (int)blockIdx.x, nr, nt, gR, gT);
    if (DBG) tk[1] = wall_clock64();
    // A segment pair holding any byte outside ACGT is left unknown: an all-N reference segment puts
    // its ~1000 identical k-mers into one LDS bucket, which every target lane hashing there scans in
    // full on each probe step (such pairs -- assembly gaps, telomeres -- took 0.2-0.8 ms per pass
    // beside the genome's other kernels).  The in-order pass classifies them when it has to.
    bool exotic = false;
    {
        const uint32_t* r4 = reinterpret_cast<const uint32_t*>(L.r);
        const uint32_t* t4 = reinterpret_cast<const uint32_t*>(L.t);
#pragma unroll
        for (int j = 0; j < SEGB / 256; j++) {
            const int i = lane + 64 * j, b0 = 4 * i;
            exotic = exotic || non_acgt4(r4[i], nr - b0) || non_acgt4(t4[i], nt - b0);
        }
        exotic = __ballot(exotic) != 0;
    }
    // The k2 hit positions decide the class of a segment pair with few of them.  Every match a pass
    // takes (compression.cpp:64-161, local: no gate) starts at a hit position, a match of length l
    // covers l - k + 1 hit positions of its diagonal, and a k-mer hit's first 10 bases are a k2 hit:
    // so either pass matches at most 14 h10 bases.  h10 = 0: neither pass finds a match (class 2 --
    // non-N: the pair is pure ACGT); 28 h10 < nt: whichever pass succeeds leaves more than half of
    // the segment literal (class 1, :417-421).  More hits: unknown (such a pair is usually aligned,
    // class 0, and no window holds it either way).  tests/test_local_proof_cpu.py checks the rule
    // against the oracle's passes.
    int c = -1, h10 = 0;
    if (!exotic) {
        seg_table<10>(L, nr);
        h10 = seg_hits<10>(L, nr, nt);
        if (h10 == 0) c = 2;
        else if (28 * h10 < nt) c = 1;
    }
    if (DBG) tk[2] = tk[3] = wall_clock64();
    if (DBG && lane == 0) {
        tk[4] = wall_clock64();
        unsigned long long* d = g_probe_dbg[blockIdx.x];
        for (int i = 0; i < 5; i++) d[i] = tk[i];
        d[5] = (unsigned long long)(c + 1) | ((unsigned long long)h10 << 8) | ((unsigned long long)seg << 32);
    }
    // (nothing else is written: a window makes the pair global, and without one the in-order pass
    // computes every segment's records, statistics and class itself)
    if (lane == 0) { pout[blockIdx.x] = c; pout[PROBE_RUNS * PROBE_RUN + blockIdx.x] = seg; }
}

__global__ void k_switch_final(const int32_t* __restrict__ cls, int32_t gen, const int64_t* __restrict__ dnR,
                               const int64_t* __restrict__ dnT, int32_t* __restrict__ ctl) {
    const int32_t nseg = seg_count(*dnR, *dnT);
    for (int32_t e = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x) + 4; e < nseg; e += (int32_t)(gridDim.x * blockDim.x)) {
        int k[5];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const int32_t t = cls[e - 4 + i];
            k[i] = (t >> 2) == gen ? (t & 3) : -1;
        }
        if (k[4] == 2 && mism(k[0]) && mism(k[1]) && mism(k[2]) && mism(k[3])) atomicMin(&ctl[2], e);
    }
}

// ---------------------------------------------------------------------------------------------
// local record text: per segment "(p,l)"/literal records, delta-encoded against the previous
// match token of the whole line (compression.cpp:258-292)
// ---------------------------------------------------------------------------------------------
__global__ void k_seg_lastkey(const SegStat* __restrict__ stat, int64_t iters, int64_t* __restrict__ v) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < iters; s += (int64_t)gridDim.x * blockDim.x)
        v[s] = (stat[s].pass && stat[s].nmatch) ? s : -1;
}

__device__ __forceinline__ int32_t prev_abs_p(const SegStat* stat, const int64_t* prevseg, int64_t s) {
    const int64_t q = prevseg[s];
    return q >= 0 ? (int32_t)(q * SEG_L + stat[q].last_p) : 0;
}

// one wave per segment: text length
__global__ __launch_bounds__(SCCG_BLOCK) void k_seg_textlen(const SegStat* __restrict__ stat, int64_t iters,
                                                            const uint32_t* __restrict__ recs,
                                                            const int64_t* __restrict__ prevseg,
                                                            int64_t* __restrict__ len, int abs_p) {
    const int64_t s = (int64_t)blockIdx.x * WPB + wave_in_block();
    if (s >= iters) return;
    const int lane = lane_id();
    const SegStat st = stat[s];
    int64_t total = 0;
    if (st.pass) {
        int32_t prev = prev_abs_p(stat, prevseg, s);
        const uint32_t* r = recs + s * SEG_REC_CAP;
        // matches need the previous token's p: do the scan in 64-record batches
        for (int b0 = 0; b0 < st.nrec; b0 += 64) {
            const int i = b0 + lane;
            const uint32_t rec = i < st.nrec ? r[i] : 0;
            const bool is_m = i < st.nrec && (rec >> 31);
            const int32_t pabs = (int32_t)(s * SEG_L) + (int32_t)((rec >> 11) & 0xfffff);
            // previous match p within the batch: last match lane before me
            const unsigned long long mm = __ballot(is_m);
            const unsigned long long before = mm & ((1ull << lane) - 1);
            const int src = before ? 63 - __clzll((long long)before) : -1;
            const int32_t pp = __shfl(pabs, src < 0 ? 0 : src, 64);
            const int32_t my_prev = abs_p ? 0 : src >= 0 ? pp : prev;
            int64_t l = 0;
            if (i < st.nrec) {
                if (is_m) l = 3 + ndigits_i32((int32_t)((uint32_t)pabs - (uint32_t)my_prev)) + ndigits_i32((int32_t)(rec & 0x7ff));
                else l = rec & 0x7ff;
            }
            total += wave_sum(l);
            if (mm) prev = __shfl(pabs, 63 - __clzll((long long)mm), 64);
        }
    }
    if (lane == 0) len[s] = total;
}

__global__ __launch_bounds__(SCCG_BLOCK) void k_seg_textwrite(const SegStat* __restrict__ stat, int64_t iters,
                                                              const uint32_t* __restrict__ recs,
                                                              const int64_t* __restrict__ prevseg,
                                                              const int64_t* __restrict__ off,
                                                              const uint8_t* __restrict__ T,
                                                              uint8_t* __restrict__ out, int abs_p) {
    __shared__ int64_t roff[WPB][64];
    const int w = wave_in_block();
    const int64_t s = (int64_t)blockIdx.x * WPB + w;
    if (s >= iters) return;
    const int lane = lane_id();
    const SegStat st = stat[s];
    if (!st.pass) return;
    int32_t prev = prev_abs_p(stat, prevseg, s);
    int64_t o = off[s];
    const uint32_t* r = recs + s * SEG_REC_CAP;
    const int64_t tbase = s * SEG_L;
    for (int b0 = 0; b0 < st.nrec; b0 += 64) {
        const int i = b0 + lane;
        const uint32_t rec = i < st.nrec ? r[i] : 0;
        const bool is_m = i < st.nrec && (rec >> 31);
        const int32_t pabs = (int32_t)(s * SEG_L) + (int32_t)((rec >> 11) & 0xfffff);
        const unsigned long long mm = __ballot(is_m);
        const unsigned long long before = mm & ((1ull << lane) - 1);
        const int src = before ? 63 - __clzll((long long)before) : -1;
        const int32_t pp = __shfl(pabs, src < 0 ? 0 : src, 64);
        const int32_t my_prev = abs_p ? 0 : src >= 0 ? pp : prev;
        const int32_t delta = (int32_t)((uint32_t)pabs - (uint32_t)my_prev);
        int64_t l = 0;
        if (i < st.nrec) l = is_m ? 3 + ndigits_i32(delta) + ndigits_i32((int32_t)(rec & 0x7ff)) : (rec & 0x7ff);
        const int64_t incl = wave_incl_add(l);
        const int64_t my_o = o + incl - l;
        if (is_m) {
            uint8_t* d = out + my_o;
            *d++ = '(';
            d += write_i32(d, delta);
            *d++ = ',';
            d += write_i32(d, (int32_t)(rec & 0x7ff));
            *d = ')';
        }
        roff[w][lane] = my_o;
        wave_sync();
        // literal runs: the whole wave copies each one
        unsigned long long lm = __ballot(i < st.nrec && !is_m);
        while (lm) {
            const int j = __ffsll((long long)lm) - 1;
            lm &= lm - 1;
            const uint32_t rj = __shfl(rec, j, 64);
            const int64_t dst = roff[w][j];
            const int start = (int)(rj >> 11), ln = (int)(rj & 0x7ff);
            for (int q = lane; q < ln; q += 64) out[dst + q] = c_toupper(T[tbase + start + q]);
        }
        wave_sync();
        o += __shfl(incl, 63, 64);
        if (mm) prev = __shfl(pabs, 63 - __clzll((long long)mm), 64);
    }
}

__global__ void k_copy_upper(const uint8_t* __restrict__ in, int64_t n, uint8_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = c_toupper(in[i]);
}

}  // namespace

int launch_local_pass(int k, int pass, int upper, const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int64_t seg0,
                      int64_t seg_end, uint32_t* recs, SegStat* stat, hipStream_t s) {
    if (seg_end <= seg0) return 0;
    unsigned g = grid_for(seg_end - seg0, WPB);
    if (g > 4096) g = 4096;
    static const bool dbg = getenv("SCCG_DEBUG") != nullptr;
    if (dbg) {
        const unsigned long long z[16] = {};
        SCCG_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_local_dbg), z, sizeof z, 0, hipMemcpyHostToDevice, s));
        SCCG_HIP(hipStreamSynchronize(s));
    }
    if (k == 14 && !dbg)
        PROF_LAUNCH(PROF_LOCAL14, s, (k_local_pass<14, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT,
                    seg0, seg_end, recs, stat);
    else if (k == 14)
        PROF_LAUNCH(PROF_LOCAL14, s, (k_local_pass<14, true>), dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT,
                    seg0, seg_end, recs, stat);
    else if (k == 10 && !dbg)
        PROF_LAUNCH(PROF_LOCAL10, s, (k_local_pass<10, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT,
                    seg0, seg_end, recs, stat);
    else if (k == 10)
        PROF_LAUNCH(PROF_LOCAL10, s, (k_local_pass<10, true>), dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT,
                    seg0, seg_end, recs, stat);
    else
        return SCCG_E_UNSUPPORTED;
    SCCG_HIP(hipGetLastError());
    if (dbg) {
        unsigned long long d[16];
        SCCG_HIP(hipMemcpyFromSymbolAsync(d, HIP_SYMBOL(g_local_dbg), sizeof d, 0, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipStreamSynchronize(s));
        const double n = d[5] ? (double)d[5] : 1.0;
        fprintf(stderr, "[local k=%d pass=%d] %llu segments, per segment (us): load %.2f keys %.2f insert %.2f hits %.2f walk %.2f"
                " | max segment %.2f\n", k, pass, d[5], d[0] / n / 100, d[1] / n / 100, d[2] / n / 100, d[3] / n / 100,
                d[4] / n / 100, d[6] / 100.0);
        fprintf(stderr, "[local]   slowest segment %llu (%llu matches): load %.1f keys %.1f hits %.1f walk %.1f us\n", d[13],
                d[14], d[8] / 100.0, (d[9] + d[10]) / 100.0, d[11] / 100.0, d[12] / 100.0);
    }
    return 0;
}

// SCCG_LOCAL_PROVE=0: every segment walks (A/B runs and tests of the proof)
int local_prove() {
    static const int v = [] { const char* e = getenv("SCCG_LOCAL_PROVE"); return e ? atoi(e) != 0 : 1; }();
    return v;
}

int launch_local_proven(const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int64_t iters, uint32_t* recs,
                        SegStat* stat, hipStream_t s) {
    if (!local_prove() || iters <= 0) return 0;
    // The k pass over the proved segments (pass 3), then k2 only over a proved segment whose k pass
    // found no match (pass 4, PASS_NEED_K2; the proof says there is none) -- not over the segments
    // k_local_all already took through both passes.
    const int rc = launch_local_pass(14, 3, 1, R, nR, T, nT, 0, iters, recs, stat, s);
    return rc ? rc : launch_local_pass(10, 4, 1, R, nR, T, nT, 0, iters, recs, stat, s);
}

int local_probe_applies(int64_t nseg_max) {
    static const bool probe_on = [] { const char* e = getenv("SCCG_SWITCH_PROBE"); return !e || atoi(e) != 0; }();
    return probe_on && nseg_max >= PROBE_MIN_SEGS;
}

int local_probe_window(const int32_t* pout) {
    int32_t best = -1;
    for (int r = 0; r < PROBE_RUNS; r++) {
        const int32_t* c = pout + r * PROBE_RUN;
        for (int i = 4; i < PROBE_RUN; i++) {
            const bool m4 = (c[i - 1] == 1 || c[i - 1] == 2) && (c[i - 2] == 1 || c[i - 2] == 2) &&
                            (c[i - 3] == 1 || c[i - 3] == 2) && (c[i - 4] == 1 || c[i - 4] == 2);
            const int32_t e = pout[PROBE_RUNS * PROBE_RUN + r * PROBE_RUN + i];
            if (c[i] == 2 && m4 && e >= 4 && (best < 0 || e < best)) best = e;
        }
    }
    return best;
}

// the probe's segments copied out of a written stripped copy (strips that wrote T / R)
__global__ void k_segment_copy(const uint8_t* __restrict__ src, const int64_t* __restrict__ d_len,
                               const int32_t* __restrict__ segs, uint8_t* __restrict__ dst) {
    const int32_t seg = segs[blockIdx.x];
    if (seg < 0) return;
    const int64_t q0 = (int64_t)seg * SEG_L, len = *d_len;
    for (int i = (int)threadIdx.x; i < SEG_L && q0 + i < len; i += (int)blockDim.x)
        dst[(size_t)blockIdx.x * SEG_GATHER_B + i] = src[q0 + i];
}

int launch_segment_copy(const uint8_t* src, const int64_t* d_len, const int32_t* segs, int nslots, uint8_t* dst,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_segment_copy, dim3(nslots), dim3(256), 0, s, src, d_len, segs, dst);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_probe_segs(const int64_t* d_nR, const int64_t* d_nT, int32_t* segs, hipStream_t s) {
    hipLaunchKernelGGL(k_probe_segs, dim3(1), dim3(PROBE_RUNS * PROBE_RUN), 0, s, d_nR, d_nT, segs);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_local_probe(const uint8_t* gR, const int64_t* d_nR, const uint8_t* gT, const int64_t* d_nT, const int32_t* segs,
                       int32_t* pout, hipStream_t s) {
    static const bool pdbg = getenv("SCCG_DEBUG") != nullptr;
    constexpr int NP = PROBE_RUNS * PROBE_RUN;
    if (!pdbg) {
        PROF_LAUNCH(PROF_LOCAL14, s, k_local_probe<false>, dim3(NP), dim3(64), 0, s, gR, d_nR, gT, d_nT, segs, pout);
    } else {
        const unsigned long long z[NP][6] = {};
        SCCG_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_probe_dbg), z, sizeof z, 0, hipMemcpyHostToDevice, s));
        PROF_LAUNCH(PROF_LOCAL14, s, k_local_probe<true>, dim3(NP), dim3(64), 0, s, gR, d_nR, gT, d_nT, segs, pout);
        unsigned long long d[NP][6];
        SCCG_HIP(hipMemcpyFromSymbolAsync(d, HIP_SYMBOL(g_probe_dbg), sizeof d, 0, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipStreamSynchronize(s));
        unsigned long long t0 = ~0ull;
        for (auto& x : d) if (x[0] && x[0] < t0) t0 = x[0];
        for (int i = 0; i < NP; i++) {
            const auto& x = d[i];
            if (!x[0]) continue;
            fprintf(stderr, "[probe] seg %llu class %d k2 hits %llu: start %.1f load %.1f end %.1f us\n",
                    x[5] >> 32, (int)(x[5] & 0xff) - 1, (x[5] >> 8) & 0xffffff, (x[0] - t0) / 100.0, (x[1] - x[0]) / 100.0,
                    (x[4] - x[0]) / 100.0);
        }
    }
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_local_all(const uint8_t* R, const int64_t* d_nR, const uint8_t* T, const int64_t* d_nT, int64_t nseg_max,
                     uint32_t* recs, SegStat* stat, int32_t* cls, int32_t gen, int32_t* ctl, hipStream_t s) {
    if (nseg_max <= 0) return 0;
    // resident capacity: the grid drains the counter, extra blocks would only find it exhausted
    static const unsigned cap = [] {
        int dev = 0, cus = 256, per = 4;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_local_all<false>, SCCG_BLOCK, 0) != hipSuccess || per < 1)
            per = 4;
        // Fewer resident blocks per CU than fit (4) leave room for the global walk's preparation and
        // round 1, which otherwise wait for the whole pass (it fills every CU's VGPRs and LDS).
        // Measured (blocks/CU 4 / 3 / 2): whole genome on 1 GPU 28.5 / 27.3 / 27.2 ms, chr1 pair
        // 1.57 / 1.55 / 1.54 ms, local-mode pair 2.84 / 2.90 / 2.97 ms.  Round 3, genome with two
        // contexts (3 / 2, interleaved, 8 pairs of runs, profiles/r03/local_bpc_ab*): 2 faster in 6 of
        // 8, medians 22.5-24.1 vs 22.3-22.4 ms -- 2 is the default.  SCCG_LOCAL_BPC overrides.
        const char* e = getenv("SCCG_LOCAL_BPC");
        const int bpc = e ? atoi(e) : 2;
        if (bpc >= 1 && bpc < per) per = bpc;
        return (unsigned)(cus * per);
    }();
    unsigned g = grid_for(nseg_max, WPB);
    if (g > cap) g = cap;
    static const bool dbg = getenv("SCCG_DEBUG") != nullptr;
    if (dbg) {
        const unsigned long long z[16] = {};
        SCCG_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_local_dbg), z, sizeof z, 0, hipMemcpyHostToDevice, s));
        PROF_LAUNCH(PROF_LOCAL14, s, k_local_all<true>, dim3(g), dim3(SCCG_BLOCK), 0, s, R, d_nR, T, d_nT, recs, stat, cls,
                    gen, ctl, local_prove());
        unsigned long long d[16];
        SCCG_HIP(hipMemcpyFromSymbolAsync(d, HIP_SYMBOL(g_local_dbg), sizeof d, 0, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipStreamSynchronize(s));
        const double n = d[5] ? (double)d[5] : 1.0;
        fprintf(stderr, "[local all] %llu segments proved class 0 without a walk\n", d[15]);
        fprintf(stderr, "[local all] %llu segment passes, per pass (us): load %.2f keys %.2f insert %.2f hits %.2f walk %.2f"
                " | max %.2f (seg %llu, %llu matches: load %.2f keys %.2f insert %.2f hits %.2f walk %.2f)\n", d[5],
                d[0] / n / 100, d[1] / n / 100, d[2] / n / 100, d[3] / n / 100, d[4] / n / 100, d[6] / 100.0, d[13], d[14],
                d[8] / 100.0, d[9] / 100.0, d[10] / 100.0, d[11] / 100.0, d[12] / 100.0);
    } else {
        PROF_LAUNCH(PROF_LOCAL14, s, k_local_all<false>, dim3(g), dim3(SCCG_BLOCK), 0, s, R, d_nR, T, d_nT, recs, stat, cls,
                    gen, ctl, local_prove());
    }
    if (nseg_max > 4) {
        const unsigned gs = grid_for(nseg_max - 4, 256) > 2048 ? 2048 : grid_for(nseg_max - 4, 256);
        hipLaunchKernelGGL(k_switch_final, dim3(gs), dim3(256), 0, s, (const int32_t*)cls, gen, d_nR, d_nT, ctl);
    }
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_local_emit(const uint8_t* T, int64_t nT, int64_t iters, const uint32_t* recs, const SegStat* stat,
                      uint8_t* out, int64_t* d_len, int64_t* d_tmp_a, int64_t* d_tmp_b, int64_t* d_partial,
                      hipStream_t s, bool abs_p) {
    // d_tmp_a: prev-match segment index, d_tmp_b: per-segment text length -> offsets
    const int64_t lead_len = iters * SEG_L < nT ? iters * SEG_L : nT;
    if (iters > 0) {
        const unsigned g = grid_for(iters, 256) > 4096 ? 4096 : grid_for(iters, 256);
        hipLaunchKernelGGL(k_seg_lastkey, dim3(g), dim3(256), 0, s, stat, iters, d_tmp_a);
        int rc = dev_excl_max(d_tmp_a, d_tmp_a, iters, nullptr, d_partial, s);
        if (rc) return rc;
        hipLaunchKernelGGL(k_seg_textlen, dim3(grid_for(iters, WPB)), dim3(SCCG_BLOCK), 0, s, stat, iters, recs,
                           (const int64_t*)d_tmp_a, d_tmp_b, (int)abs_p);
        rc = dev_excl_sum(d_tmp_b, d_tmp_b, iters, d_len, d_partial, s);
        if (rc) return rc;
        PROF_LAUNCH(PROF_LOCAL_EMIT, s, k_seg_textwrite, dim3(grid_for(iters, WPB)), dim3(SCCG_BLOCK), 0, s, stat, iters, recs,
                           (const int64_t*)d_tmp_a, (const int64_t*)d_tmp_b, T, out, (int)abs_p);
        SCCG_HIP(hipGetLastError());
    } else {
        SCCG_HIP(hipMemsetAsync(d_len, 0, sizeof(int64_t), s));
    }
    // leftover target segments (compression.cpp:476-481) go after the segment text
    int64_t seg_text = 0;
    {
        const RbItem it{d_len, &seg_text, (int)sizeof seg_text};
        const int rc = dev_readback(&it, 1, s);
        if (rc) return rc;
    }
    const int64_t rest = nT - lead_len;
    if (rest > 0) {
        const unsigned g = grid_for(rest, 256) > 8192 ? 8192 : grid_for(rest, 256);
        hipLaunchKernelGGL(k_copy_upper, dim3(g), dim3(256), 0, s, T + lead_len, rest, out + seg_text);
        SCCG_HIP(hipGetLastError());
    }
    const int64_t total = seg_text + (rest > 0 ? rest : 0);
    return dev_set_i64(d_len, 1, {total}, s);
}
