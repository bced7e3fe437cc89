// ingest.hip -- FASTA strip, byte filters, run extraction and run-line text.
//
// Everything here is HBM-bound byte work: one 8 KiB tile per 256-thread block (32 bytes per
// thread), reduce-then-scan for the output offsets, no atomics on the data path.
//
//   read_genomes_from_files  compression.cpp:181-220 (decompression.cpp:47-58 for the reference)
//   lowercase / N run lines  compression.cpp:341-368, :495-522, :527-555
//   N erase + toupper        compression.cpp:369-370, :523-524, :556-557; decompression.cpp:105-110
#include "internal.h"

namespace {

constexpr int PER_T = INGEST_TILE / SCCG_BLOCK;  // 32 bytes per thread
constexpr int WPB = SCCG_BLOCK / 64;             // wave tiles per block

// ---------------------------------------------------------------------------------------------
// header search
// ---------------------------------------------------------------------------------------------

// First position >= from (from = *from_slot + 1, or 0) holding `c` (mode 1) or a '>' that starts a
// line (mode 0).  Blocks take 16 KiB chunks in increasing order from a ticket and stop as soon as a
// chunk starts past the best match: a header at the start of the file costs one wave of chunks,
// not a pass over the whole FASTA.  Every thread loads its 64 bytes at once (a byte loop with an
// early exit issues its loads one after another: ~50 us behind a busy HBM).  *res must hold n on
// entry; *ticket 0.
constexpr int64_t FM_CHUNK = 16384;
template <int NW>
__device__ __forceinline__ uint8_t wb(const uint32_t (&w)[NW], int i) { return (uint8_t)(w[i >> 2] >> (8 * (i & 3))); }
template <int NW>
__device__ __forceinline__ void load_words(const uint8_t* __restrict__ buf, int64_t n, int64_t off, uint32_t (&w)[NW]);
__global__ __launch_bounds__(SCCG_BLOCK) void k_first_match(const uint8_t* __restrict__ buf, int64_t n,
                                                            const int64_t* __restrict__ from_slot, int mode, uint8_t c,
                                                            int64_t* __restrict__ res, unsigned int* __restrict__ ticket) {
    __shared__ int64_t s_cs;
    const int64_t from = from_slot ? *from_slot + 1 : 0;
    const int64_t base = from & ~(int64_t)63;   // chunks start 64-byte aligned; bytes before `from` are skipped
    constexpr int PER = FM_CHUNK / SCCG_BLOCK;   // 64 bytes per thread
    for (;;) {
        if (threadIdx.x == 0) {
            const int64_t cs = base + (int64_t)atomicAdd(ticket, 1u) * FM_CHUNK;
            const int64_t best = (int64_t)__hip_atomic_load((unsigned long long*)res, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_cs = (cs >= n || cs >= best) ? -1 : cs;
        }
        __syncthreads();
        const int64_t cs = s_cs;
        __syncthreads();
        if (cs < 0) return;
        const int64_t p0 = cs + (int64_t)threadIdx.x * PER;
        // (no `continue` past the barriers above: lanes of one wave would then reach them in
        // different iterations, and the block deadlocks)
        if (p0 < n) {
            uint32_t w[PER / 4];
            load_words<PER / 4>(buf, n, p0, w);
            uint8_t prev = p0 > 0 ? buf[p0 - 1] : (uint8_t)'\n';
            int64_t hit = INT64_MAX;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const uint8_t b = wb(w, i);
                const int64_t p = p0 + i;
                const bool ok = p >= from && p < n && (mode == 0 ? (b == '>' && (p == 0 || prev == '\n')) : (b == c));
                if (ok && hit == INT64_MAX) hit = p;
                prev = b;
            }
            if (hit != INT64_MAX) atomicMin((unsigned long long*)res, (unsigned long long)hit);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// FASTA strip (+ optional byte filter in the same pass).  A line's fate is decided by its first
// byte (REF: '>' lines dropped; TGT: only the header line [h, he) dropped); every isspace byte is
// dropped.  In REF mode bytes before the first line start of a tile inherit the status of an
// earlier tile: the per-tile summary keeps those bytes apart (a) from the ones whose status is
// known (b).  The filter output (N erase + toupper) is the filter applied to the strip output, so
// it carries the same (a, b) split (fa, fb).
//
// A tile is one wave's 4 KiB (64 bytes per lane): summary and write need wave operations only, no
// workgroup barrier, so every wave streams on its own.  Writes are staged: every lane drops its
// kept bytes into the wave's LDS copy of the tile's output at its wave-scan offset, then the wave
// stores the tile's output range with aligned dword stores.
// ---------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void load_words(const uint8_t* __restrict__ buf, int64_t n, int64_t off, uint32_t (&w)[NW]) {
    if (off + 4 * NW <= n && (((uintptr_t)(buf + off)) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(buf + off);
#pragma unroll
        for (int q = 0; q < NW / 4; q++) {
            const uint4 v = p[q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < NW; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int64_t p = off + 4 * q + i;
                v |= (uint32_t)(p < n ? buf[p] : (uint8_t)' ') << (8 * i);
            }
            w[q] = v;
        }
    }
}

__device__ __forceinline__ bool filter_keep(FilterMode m, uint8_t c) {
    if (m == FILTER_DROP_N_UPPER) return c != 'N' && c != 'n';
    if (m == FILTER_DROP_UPPERN_ONLY) return c != 'N';
    return true;
}

// SWAR byte tests on 4 bytes: bit 7 of each byte set where the test holds
__device__ __forceinline__ uint32_t sw_lt(uint32_t x, uint32_t n) {   // byte < n, n <= 128
    return ~(((x & 0x7F7F7F7Fu) + (0x80u - n) * 0x01010101u) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t sw_eq(uint32_t x, uint32_t c) { return sw_lt(x ^ (c * 0x01010101u), 1); }
__device__ __forceinline__ uint32_t sw_bits(uint32_t hm) { return ((hm >> 7) * 0x01020408u) >> 24; }   // -> 4 bits
// toupper of 4 bytes
__device__ __forceinline__ uint32_t sw_upper(uint32_t x) {
    const uint32_t lower = sw_lt(x, 'z' + 1) & ~sw_lt(x, 'a');
    return x - (lower >> 2);
}

template <bool UP>
__device__ __forceinline__ uint8_t up_byte(uint8_t c) { return UP && c >= 'a' && c <= 'z' ? (uint8_t)(c - 32) : c; }

constexpr int SL = 64;                 // strip bytes per lane
constexpr int SNW = SL / 4;            // words per lane
constexpr int STRIP_WTILE = 64 * SL;   // bytes per wave tile
static_assert(STRIP_WTILE == STRIP_TILE, "tile size shared with the host");

// LDS staging of a wave tile's output, in output order.  Each lane compacts its 64 bytes a word
// at a time: v_perm packs a word's kept bytes to the low end (selector from a 16-entry table by
// the word's 4-bit keep mask) into a 64-bit accumulator aligned to the stage's dwords, and every
// completed dword is stored with an aligned ds_write_b32 (unaligned LDS stores stall).  A lane's
// first dword may start with bytes of earlier lanes (written as garbage here) and its last bytes
// may share a dword with later lanes: after all dword stores, every lane stores its final partial
// dword byte by byte, which also repairs the garbage that later lanes put there.
constexpr int STAGE_WORDS = STRIP_WTILE / 4 + 2;
__device__ __forceinline__ uint32_t stage_word(const uint32_t* st4, int d) { return st4[d]; }

// Wave store of the `cnt` staged bytes to out[g0, g0 + cnt): head bytes up to a 16-byte boundary,
// a 16-byte body (one dwordx4 store per lane and 1 KiB, four times fewer store instructions than
// dword stores), tail bytes.  The body's byte shift against the stage is the same for every lane.
// UP: uppercased on the way out (the filtered copy of a wave tile whose filter dropped nothing).
template <bool UP = false>
__device__ __forceinline__ void stage_out(const uint32_t* __restrict__ st4, int cnt, uint8_t* __restrict__ out, int64_t g0) {
    const uint8_t* st = reinterpret_cast<const uint8_t*>(st4);
    const int t = lane_id();
    int head = (int)((16 - (((uintptr_t)(out + g0)) & 15)) & 15);
    if (head > cnt) head = cnt;
    if (t < head) out[g0 + t] = up_byte<UP>(st[t]);
    const int n16 = (cnt - head) >> 4;
    const uint32_t sh = (uint32_t)(head & 3);
    uint4* o16 = reinterpret_cast<uint4*>(out + g0 + head);
    for (int d = t; d < n16; d += 64) {
        const int b = (head >> 2) + 4 * d;   // (the last word read: <= cnt / 4 < STAGE_WORDS)
        const uint32_t w0 = stage_word(st4, b), w1 = stage_word(st4, b + 1), w2 = stage_word(st4, b + 2),
                       w3 = stage_word(st4, b + 3), w4 = stage_word(st4, b + 4);
        uint4 v = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                             __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
        if (UP) v = make_uint4(sw_upper(v.x), sw_upper(v.y), sw_upper(v.z), sw_upper(v.w));
        o16[d] = v;
    }
    const int done = head + 16 * n16;
    if (t < cnt - done) out[g0 + done + t] = up_byte<UP>(st[done + t]);
}

// v_perm selectors: kept bytes of a word (4-bit mask) to the low end, zeros above (0x0c)
__device__ __forceinline__ uint32_t compact_sel(uint32_t m) {
    uint32_t sel = 0x0c0c0c0cu;
    int k = 0;
    for (int i = 0; i < 4; i++)
        if ((m >> i) & 1u) { sel = (sel & ~(0xffu << (8 * k))) | ((uint32_t)i << (8 * k)); k++; }
    return sel;
}

// Stage the bytes of w (uppercased if UP) selected by keep at byte q0 of st (the lane's output
// offset in the tile).
template <bool UP>
__device__ __forceinline__ void stage_lane(uint8_t* __restrict__ st, const uint32_t* __restrict__ tab,
                                           const uint32_t (&w)[SNW], uint64_t keep, int q0) {
    const int mis = q0 & 3;
    uint32_t* const a0 = reinterpret_cast<uint32_t*>(st + (q0 - mis));
    uint32_t* a4 = a0;
    uint64_t acc = 0;
    int an = mis;   // bytes in acc (the first `mis` belong to earlier lanes)
#pragma unroll
    for (int h = 0; h < SNW; h += 8) {
        uint32_t sel[8];   // selectors first: a table read behind the stage writes would wait for them
#pragma unroll
        for (int j = 0; j < 8; j++) sel[j] = tab[(uint32_t)(keep >> (4 * (h + j))) & 0xfu];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t m = (uint32_t)(keep >> (4 * (h + j))) & 0xfu;
            const uint32_t x = UP ? sw_upper(w[h + j]) : w[h + j];
            acc |= (uint64_t)__builtin_amdgcn_perm(0u, x, sel[j]) << (8 * an);
            an += __builtin_popcount(m);
            if (an >= 4) {
                *a4++ = (uint32_t)acc;
                acc >>= 32;
                an -= 4;
            }
        }
    }
    wave_sync();
    uint8_t* tb = reinterpret_cast<uint8_t*>(a4);
#pragma unroll
    for (int i = 0; i < 3; i++)
        if (i < an && (a4 != a0 || i >= mis)) tb[i] = (uint8_t)(acc >> (8 * i));
}

// Per-lane byte masks of a 64-byte range (bit i = byte off + i):
//   known    kept by strip, line status decided inside the range (REF) / always (TGT)
//   unknown  REF: non-space bytes before the range's first line start (status from earlier)
//   fk       kept by the byte filter;  par  '(' bytes
struct StripMasks {
    uint64_t known, unknown, fk, par;
    int32_t last;   // status of the last line start in range: -1 none, 0 drop, 1 keep
    uint64_t lower, nn;   // RUNS: bytes 'a'..'z' and bytes 'N' / 'n' (the two run lines' predicates)
    uint64_t odd;         // ODD: nonzero when a flagged byte is neither whitespace nor a letter other than N / n
};

// RUNS: lowercase bytes by bit 5 alone -- exact for letters (and unkept whitespace does not matter)
__device__ __forceinline__ uint64_t lower_fast(const uint32_t (&w)[SNW]) {
    uint64_t lo = 0;
#pragma unroll
    for (int q = 0; q < SNW; q++) {
        const uint32_t t = (w[q] >> 5) & 0x01010101u;
        lo |= (uint64_t)(((t * 0x01020408u) >> 24) & 0xfu) << (4 * q);
    }
    return lo;
}

__device__ __forceinline__ uint64_t below64(int k) { return k >= 64 ? ~0ull : (1ull << k) - 1ull; }

template <IngestMode MODE, bool RUNS = false, bool ODD = false>
__device__ __forceinline__ StripMasks strip_masks(FilterMode fm, const uint32_t (&w)[SNW], uint8_t prev, int64_t off,
                                                  int64_t n, int64_t h, int64_t he, const uint8_t* __restrict__ lbytes) {
    // Byte classes.  Every byte that matters (whitespace, '\n', '>', '(', N / n) is outside
    // {A,C,G,T,a,c,g,t}, which one 2-bit-code round trip per word flags (on the word with bit 5
    // cleared: the case fold); only the flagged bytes -- a line's '\n' per ~60 bases, N runs -- are
    // classified, one at a time from the lane's LDS copy (lbytes).  (Classifying every byte with
    // SWAR compares cost ~45 VALU per word: the strip kernels were VALU-bound.)
    // The flags are gathered interleaved (cheaper than packing each word's 4 bits in order): bit
    // 32h + 8b + r of sp flags byte 32h + 4r + b (word 8h + r, byte b of it).
    uint32_t sph[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        uint32_t x = 0;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            uint32_t d;
            (void)swar_codes(w[8 * h + r] & 0xDFDFDFDFu, d);
            const uint32_t hm = ((((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d) & 0x80808080u);   // bit 7: byte != 0
            x |= hm >> (7 - r);
        }
        sph[h] = x;
    }
    const uint64_t sp = ((uint64_t)sph[1] << 32) | sph[0];
    // RUNS: lowercase bytes in byte order -- an unflagged byte (A C G T a c g t) is lowercase iff its
    // bit 5 is set (a word's four bits gathered by one multiply); flagged bytes are set below
    uint64_t lo = RUNS ? lower_fast(w) : 0ull, nn = 0;
    uint64_t ws = 0, nl = 0, gt = 0, drop = 0, par = 0;
    bool odd = false;   // (a lane flag: its compares stay in scalar lane masks)
    for (uint64_t m = sp; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        const int i = (j & 32) + 4 * (j & 7) + ((j >> 3) & 3);
        const uint32_t c = lbytes[i];
        const uint64_t bit = 1ull << i;
        if (RUNS) {
            lo &= ~bit;
            if (c >= 'a' && c <= 'z') lo |= bit;
            if (c == 'N' || c == 'n') nn |= bit;
        }
        const bool space = c == ' ' || (c >= 9 && c <= 13);
        if (space) ws |= bit;   // isspace
        if (ODD) {   // (bitwise, not short-circuit: a branch per flagged byte cost more than the compares)
            const uint32_t cl = c | 32u;
            odd |= !(space | (((cl - 'a') < 26u) & (cl != 'n')));
        }
        if (MODE == INGEST_REF) {
            if (c == '\n') nl |= bit;
            if (c == '>') gt |= bit;
        }
        if ((c == 'N' && fm != FILTER_UPPER) || (c == 'n' && fm == FILTER_DROP_N_UPPER)) drop |= bit;
        if (c == '(') par |= bit;
    }
    const uint64_t fk = ~drop;
    const int64_t lim = n - off;
    const uint64_t valid = lim >= 64 ? ~0ull : (lim > 0 ? (1ull << lim) - 1ull : 0ull);
    StripMasks r{0, 0, fk, par, -1, lo, nn, odd ? 1ull : 0ull};
    if (MODE == INGEST_TGT) {
        const int64_t lo = h - off < 0 ? 0 : (h - off > 64 ? 64 : h - off);
        const int64_t hi = he - off < 0 ? 0 : (he - off > 64 ? 64 : he - off);
        r.known = ~ws & valid & ~(below64((int)hi) & ~below64((int)lo));
        return r;
    }
    // REF: a line's fate is its first byte; line starts are position 0 and bytes after a '\n'
    const uint64_t ls = ((nl << 1) | (uint64_t)(off == 0 || prev == '\n')) & valid;
    const int first = ls ? __builtin_ctzll(ls) : 64;
    r.unknown = ~ws & valid & below64(first);
    uint64_t keep = 0;
    if ((gt & ls) == 0) {   // no '>' line here: everything from the first line start on is kept
        keep = ~below64(first);
        r.last = ls ? 1 : -1;
    } else {
        uint64_t rem = ls;
        while (rem) {
            const int j = __builtin_ctzll(rem);
            rem &= rem - 1;
            const int nx = rem ? __builtin_ctzll(rem) : 64;
            const int32_t st = !((gt >> j) & 1ull);
            if (st) keep |= below64(nx) & ~below64(j);
            r.last = st;
        }
    }
    r.known = ~ws & valid & keep;
    return r;
}

// A lane's 64 bytes of a wave tile.  Loaded coalesced (SCCG_STRIP_COALESCED, default): load q of the
// wave reads the tile's q-th KiB, 16 bytes per lane in lane order (8 cache lines per instruction,
// against 32 when every lane reads its own 64 contiguous bytes), through the wave's 4 KiB of LDS,
// from which every lane reads back its 64 contiguous bytes.
#ifndef SCCG_STRIP_COALESCED
#define SCCG_STRIP_COALESCED 0
#endif
__device__ __forceinline__ void load_lane64(const uint8_t* __restrict__ buf, int64_t n, int64_t off, uint4* __restrict__ tin,
                                            uint32_t (&w)[SNW]) {
    const int lane = lane_id();
    const int64_t t0 = off - (int64_t)lane * SL;   // the wave tile's first byte
    if (SCCG_STRIP_COALESCED && tin && t0 + STRIP_WTILE <= n && (((uintptr_t)(buf + t0)) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(buf + t0);
        uint4 v[SNW / 4];
#pragma unroll
        for (int q = 0; q < SNW / 4; q++) v[q] = p[64 * q + lane];
        wave_sync();   // (the previous user of tin is done)
#pragma unroll
        for (int q = 0; q < SNW / 4; q++) tin[64 * q + lane] = v[q];
        wave_sync();
#pragma unroll
        for (int q = 0; q < SNW / 4; q++) {
            const uint4 x = tin[4 * lane + q];
            w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
        }
        wave_sync();   // tin is free again (k_strip_write stages its output there)
    } else {
        load_words<SNW>(buf, n, off, w);
    }
}

// A wave's tile: its words, the byte before it (lane 0's 'prev'), the masks, and each lane's prior
// line status inside the wave (-1: no line start in the lanes before it).
template <IngestMode MODE, bool RUNS = false, bool ODD = false>
__device__ __forceinline__ StripMasks strip_tile(FilterMode fm, const uint8_t* __restrict__ buf, int64_t n, int64_t h,
                                                 int64_t he, int64_t off, uint32_t (&w)[SNW], int32_t& prior,
                                                 uint64_t& lsm, uint4* tin) {
    const int lane = lane_id();
    load_lane64(buf, n, off, tin, w);
    // the lane's 64 bytes in the wave's LDS buffer, for strip_masks' byte lookups (the coalesced
    // load leaves them there already, in the same layout)
    if (!(SCCG_STRIP_COALESCED && tin && off - (int64_t)lane * SL + STRIP_WTILE <= n &&
          (((uintptr_t)(buf + off - (int64_t)lane * SL)) & 15) == 0)) {
        wave_sync();
#pragma unroll
        for (int q = 0; q < SNW / 4; q++) tin[4 * lane + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        wave_sync();
    }
    uint8_t prev = '\n';
    if (MODE == INGEST_REF) {
        const uint32_t up = (uint32_t)__shfl_up((int)w[SNW - 1], 1, 64) >> 24;
        prev = lane ? (uint8_t)up : ((off > 0 && off - 1 < n) ? buf[off - 1] : (uint8_t)'\n');
    }
    const StripMasks r = strip_masks<MODE, RUNS, ODD>(fm, w, prev, off, n, h, he, reinterpret_cast<const uint8_t*>(tin + 4 * lane));
    wave_sync();   // (k_strip_write stages its output in tin next)
    prior = -1;
    lsm = 0;
    if (MODE == INGEST_REF) {
        lsm = __ballot(r.last >= 0);
        const uint64_t m = lsm & below64(lane);
        const int src = m ? 63 - __builtin_clzll(m) : 0;
        const int32_t v = __shfl(r.last, src, 64);
        prior = m ? v : -1;
    }
    return r;
}

// KC: also the keep-mask cache of the write pass.  kc: per lane the positions of its (at most two)
// unkept bytes, 7 bits each (64: none), with the tile's line status assumed "keep" where it is
// still open -- a FASTA line of 32 or more bytes leaves one or two newlines per 64-byte lane.
// kflag bit 0: the tile is plain -- every byte outside ACGTacgt is whitespace or a letter other
// than N / n (nothing is filtered, no '(' or '>' is kept, the run predicates follow from the bytes
// alone) and no lane has more than two unkept bytes; bit 1: some kept byte depends on the line
// status carried in from earlier tiles.
template <IngestMode MODE, bool KC>
__global__ __launch_bounds__(SCCG_BLOCK) void k_strip_summary(FilterMode fm, const uint8_t* __restrict__ buf, int64_t n,
                                                              const int64_t* __restrict__ hdr, int64_t* __restrict__ ta,
                                                              int64_t* __restrict__ tb, int64_t* __restrict__ tfa,
                                                              int64_t* __restrict__ tfb, int32_t* __restrict__ tlast,
                                                              uint16_t* __restrict__ kc, int32_t* __restrict__ kflag) {
    __shared__ uint4 tin_all[WPB][STRIP_WTILE / 16];
    const int64_t tile = (int64_t)blockIdx.x * WPB + wave_in_block();
    if (tile * STRIP_WTILE >= n) return;
    const int lane = lane_id();
    const int64_t off = tile * STRIP_WTILE + (int64_t)lane * SL;
    const int64_t h = MODE == INGEST_TGT ? hdr[0] : 0, he = MODE == INGEST_TGT ? hdr[1] : 0;
    uint32_t w[SNW];
    int32_t prior;
    uint64_t lsm;
    const StripMasks r = strip_tile<MODE, false, KC>(fm, buf, n, h, he, off, w, prior, lsm, tin_all[wave_in_block()]);
    if (KC) {
        const uint64_t hole = ~(r.known | (prior != 0 ? r.unknown : 0ull));
        const uint32_t h1 = hole ? (uint32_t)__builtin_ctzll(hole) : 64u, h2 = hole ? 63u - (uint32_t)__builtin_clzll(hole) : 64u;
        kc[tile * 64 + lane] = (uint16_t)(h1 | (h2 << 7));
        const uint64_t odd = __ballot(r.odd != 0 || __popcll(hole) > 2);
        const uint64_t sens = __ballot(MODE == INGEST_REF && prior < 0 && r.unknown != 0);
        if (lane == 0) kflag[tile] = (odd ? 0 : 1) | (sens ? 2 : 0);
    }
    // a-bytes of a lane with a prior line start in the wave are resolved now
    const uint64_t ra = (uint64_t)__popcll(r.unknown), rb = (uint64_t)__popcll(r.known);
    const uint64_t rfa = (uint64_t)__popcll(r.unknown & r.fk), rfb = (uint64_t)__popcll(r.known & r.fk);
    const uint64_t A = prior < 0 ? ra : 0, B = rb + (prior == 1 ? ra : 0);
    const uint64_t FA = prior < 0 ? rfa : 0, FB = rfb + (prior == 1 ? rfa : 0);
    // (each field's total <= 4096: the two 32-bit halves are summed apart)
    const uint32_t t_ab = lane_val(wave_incl_add_dpp((uint32_t)(A | (B << 16))), 63);
    const uint32_t t_f = lane_val(wave_incl_add_dpp((uint32_t)(FA | (FB << 16))), 63);
    const uint64_t tot = (uint64_t)t_ab | ((uint64_t)t_f << 32);
    if (lane == 0) {
        ta[tile] = (int64_t)(tot & 0xffff);
        tb[tile] = (int64_t)((tot >> 16) & 0xffff);
        tfa[tile] = (int64_t)((tot >> 32) & 0xffff);
        tfb[tile] = (int64_t)(tot >> 48);
    }
    if (MODE == INGEST_REF) {
        const int32_t last = lsm ? __shfl(r.last, 63 - __builtin_clzll(lsm), 64) : -1;
        if (lane == 0) tlast[tile] = last;
    } else if (lane == 0) {
        tlast[tile] = -1;
    }
}

// Tile summary monoid: (a, b, fa, fb, last), "X then Y": Y's status-unknown bytes are resolved by
// X's last line status (kept if 1, dropped if 0, still unknown if X has no line start).
struct TileSum {
    int64_t a, b, fa, fb;
    int32_t last;
};
__device__ __forceinline__ TileSum ts_compose(const TileSum& x, const TileSum& y) {
    TileSum r;
    r.a = x.a + (x.last < 0 ? y.a : 0);
    r.b = x.b + y.b + (x.last == 1 ? y.a : 0);
    r.fa = x.fa + (x.last < 0 ? y.fa : 0);
    r.fb = x.fb + y.fb + (x.last == 1 ? y.fa : 0);
    r.last = y.last >= 0 ? y.last : x.last;
    return r;
}
__device__ __forceinline__ TileSum ts_shfl_up(const TileSum& v, int d) {
    TileSum r;
    r.a = __shfl_up(v.a, d, 64); r.b = __shfl_up(v.b, d, 64);
    r.fa = __shfl_up(v.fa, d, 64); r.fb = __shfl_up(v.fb, d, 64);
    r.last = __shfl_up(v.last, d, 64);
    return r;
}

// Scan of the tile summaries in three launches.  (1) one thread per tile, 1024 tiles per block:
// block-local exclusive prefix, written over the tile's own summary, and the block total;
// (2) one block: exclusive prefix of the block totals; (3) per tile: stream prefix = "carry 1"
// then block prefix then local prefix -> output offsets (strip and filter) and carry-in status.
constexpr int SCAN_B = 1024;
__device__ __forceinline__ TileSum block_scan_tiles(TileSum v, TileSum* wsum, TileSum* total) {
    const TileSum id{0, 0, 0, 0, -1};
    const int lane = lane_id(), w = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6);
    TileSum incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const TileSum o = ts_shfl_up(incl, d);
        if (lane >= d) incl = ts_compose(o, incl);
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        TileSum run = id;
        for (int i = 0; i < nw; i++) { const TileSum x = wsum[i]; wsum[i] = run; run = ts_compose(run, x); }
        wsum[16] = run;
    }
    __syncthreads();
    TileSum ex = ts_shfl_up(incl, 1);
    if (lane == 0) ex = id;
    if (total) *total = wsum[16];
    return ts_compose(wsum[w], ex);
}

// (SCCG_SCAN_T threads per block, SCAN_B / SCAN_T tiles per thread.  A 1024-thread block waits for
// a whole free CU -- the target's scan sat ~140 us behind the reference strip's write pass on the
// side stream in a chr1 trace -- but 256-thread builds measured within noise end to end.)
#ifndef SCCG_SCAN_T
#define SCCG_SCAN_T 1024
#endif
constexpr int SCAN_T = SCCG_SCAN_T, SCAN_PER = SCAN_B / SCAN_T;
__global__ __launch_bounds__(SCAN_T) void k_strip_scan_local(int64_t ntiles, int64_t* __restrict__ ta, int64_t* __restrict__ tb,
                                                          int64_t* __restrict__ tfa, int64_t* __restrict__ tfb,
                                                          int32_t* __restrict__ tlast, TileSum* __restrict__ btot) {
    __shared__ TileSum wsum[17];
    const TileSum id{0, 0, 0, 0, -1};
    const int64_t t0 = (int64_t)blockIdx.x * SCAN_B + (int64_t)threadIdx.x * SCAN_PER;
    TileSum v[SCAN_PER], agg = id;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        const int64_t t = t0 + k;
        v[k] = t < ntiles ? TileSum{ta[t], tb[t], tfa[t], tfb[t], tlast[t]} : id;
        agg = ts_compose(agg, v[k]);
    }
    TileSum tot;
    TileSum run = block_scan_tiles(agg, wsum, &tot);
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        const int64_t t = t0 + k;
        if (t < ntiles) { ta[t] = run.a; tb[t] = run.b; tfa[t] = run.fa; tfb[t] = run.fb; tlast[t] = run.last; }
        run = ts_compose(run, v[k]);
    }
    if (threadIdx.x == 0) btot[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void k_strip_scan_blocks(int64_t nblk, TileSum* __restrict__ btot) {
    __shared__ TileSum wsum[17];
    const TileSum id{0, 0, 0, 0, -1};
    const int64_t i0 = (int64_t)threadIdx.x * SCAN_PER;
    TileSum v[SCAN_PER], agg = id;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        v[k] = i0 + k < nblk ? btot[i0 + k] : id;
        agg = ts_compose(agg, v[k]);
    }
    TileSum tot;
    TileSum run = block_scan_tiles(agg, wsum, &tot);
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        if (i0 + k < nblk) btot[i0 + k] = run;
        run = ts_compose(run, v[k]);
    }
    if (threadIdx.x == 0) btot[SCAN_B] = tot;
}

__global__ void k_strip_scan_apply(int64_t ntiles, const int64_t* __restrict__ ta, const int64_t* __restrict__ tb,
                                   const int64_t* __restrict__ tfa, const int64_t* __restrict__ tfb,
                                   const int32_t* __restrict__ tlast, const TileSum* __restrict__ btot,
                                   int64_t* __restrict__ toff, int64_t* __restrict__ toff2, int32_t* __restrict__ tcarry,
                                   int64_t* __restrict__ d_len, int64_t* __restrict__ d_len2) {
    const TileSum start{0, 0, 0, 0, 1};   // the stream starts as if after a kept line
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
        const TileSum r = ts_compose(ts_compose(start, btot[t / SCAN_B]), TileSum{ta[t], tb[t], tfa[t], tfb[t], tlast[t]});
        toff[t] = r.b;
        toff2[t] = r.fb;
        tcarry[t] = r.last;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const TileSum r = ts_compose(start, btot[SCAN_B]);
        *d_len = r.b;
        if (d_len2) *d_len2 = r.fb;
    }
}

// Run events of a lane's kept bytes (RUNS: the target strip emits both run lines' boundaries,
// compression.cpp:341-368 lowercase and :527-555 N, instead of two more passes over T).  For a
// predicate mask p (byte order) and the kept bytes K, the predicate of "the previous kept byte" at
// every position is p on K filled forward over the dropped bytes D (newlines) -- one carry trick:
// a D run that starts right after a kept 1 is the set of D bits the +s carry clears.  A run starts
// at a kept byte whose predicate holds and whose previous kept byte's does not, and ends (exclusive)
// at a kept byte where it is the other way round.  cin: the previous kept byte's predicate.
__device__ __forceinline__ void run_events(uint64_t p, uint64_t K, uint32_t cin, uint64_t& st, uint64_t& en) {
    const uint64_t D = ~K;
    const uint64_t x = p & K;
    const uint64_t sd = ((x << 1) | cin) & D;
    const uint64_t g = x | (D & ~(D + sd));
    const uint64_t prev = (g << 1) | cin;
    st = K & g & ~prev;
    en = K & ~g & prev;
}

template <IngestMode MODE, bool RUNS>
__global__ __launch_bounds__(SCCG_BLOCK) void k_strip_write(FilterMode fm, const uint8_t* __restrict__ buf, int64_t n,
                                                            const int64_t* __restrict__ hdr,
                                                            const int64_t* __restrict__ toff,
                                                            const int64_t* __restrict__ toff2,
                                                            const int32_t* __restrict__ tcarry,
                                                            uint8_t* __restrict__ out, uint8_t* __restrict__ out2,
                                                            int32_t* __restrict__ flags, RunSlots rsl,
                                                            const uint16_t* __restrict__ kc, const int32_t* __restrict__ kflag) {
    __shared__ uint4 stage_all4[WPB][(STAGE_WORDS + 3) / 4];   // (also the coalesced load's transpose)
    __shared__ uint32_t tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = compact_sel(threadIdx.x);
    __syncthreads();
    const int64_t tile = (int64_t)blockIdx.x * WPB + wave_in_block();
    if (tile * STRIP_WTILE >= n) return;
    const int lane = lane_id();
    uint32_t* st4 = reinterpret_cast<uint32_t*>(stage_all4[wave_in_block()]);
    uint8_t* s1 = reinterpret_cast<uint8_t*>(st4);
    const int64_t off = tile * STRIP_WTILE + (int64_t)lane * SL;
    const int64_t h = MODE == INGEST_TGT ? hdr[0] : 0, he = MODE == INGEST_TGT ? hdr[1] : 0;
    uint32_t w[SNW];
    int32_t prior;
    uint64_t lsm;
    StripMasks r;
    // a plain tile (k_strip_summary's kflag) takes its kept bytes from the summary's mask cache
    // instead of classifying its bytes again, unless they depend on a carried-in line status other
    // than "keep"
    const int32_t kf = kc ? uni(kflag[tile]) : 0;
    if ((kf & 1) && (MODE == INGEST_TGT || !(kf & 2) || uni(tcarry[tile]) == 1)) {
        load_words<SNW>(buf, n, off, w);
        const uint32_t code = kc[tile * 64 + lane], h1 = code & 127u, h2 = code >> 7;
        const uint64_t keep = ~((h1 < 64 ? 1ull << h1 : 0ull) | (h2 < 64 ? 1ull << h2 : 0ull));
        r = StripMasks{keep, 0ull, ~0ull, 0ull, -1, RUNS ? lower_fast(w) : 0ull, 0ull, 0ull};
        prior = 1;
    } else {
        r = strip_tile<MODE, RUNS>(fm, buf, n, h, he, off, w, prior, lsm, stage_all4[wave_in_block()]);
        if (MODE == INGEST_REF && prior < 0) prior = tcarry[tile];
    }
    const uint64_t keep = r.known | (prior == 1 ? r.unknown : 0ull), fkeep = keep & r.fk;
    const uint32_t c = (uint32_t)__popcll(keep) | ((uint32_t)__popcll(fkeep) << 16);
    const uint32_t incl = wave_incl_add_dpp(c), tot = lane_val(incl, 63);
    const uint32_t ex = incl - c;
    if (RUNS) {
        // the previous kept byte's predicates: the nearest earlier lane with a kept byte; the wave's
        // first such lane takes its own first byte's (no event there -- the tile boundary is settled
        // by k_runs_tiles from the tile's first/last predicates)
        const bool has = keep != 0;
        const int fb = has ? __builtin_ctzll(keep) : 0, lb = has ? 63 - __builtin_clzll(keep) : 0;
        const uint32_t first2 = (uint32_t)((r.lower >> fb) & 1u) | ((uint32_t)((r.nn >> fb) & 1u) << 1);
        const uint32_t last2 = (uint32_t)((r.lower >> lb) & 1u) | ((uint32_t)((r.nn >> lb) & 1u) << 1);
        const uint64_t hm = __ballot(has);
        const uint64_t before = hm & below64(lane);
        const int src = before ? 63 - __builtin_clzll(before) : 0;
        const uint32_t pl = (uint32_t)__shfl((int)last2, src, 64);
        const uint32_t cin = before ? pl : first2;
        uint64_t sl = 0, el = 0, sn = 0, en = 0;
        if (has) {
            run_events(r.lower, keep, cin & 1u, sl, el);
            run_events(r.nn, keep, cin >> 1, sn, en);
        }
        const uint64_t cc = (uint64_t)__popcll(sl) | ((uint64_t)__popcll(el) << 16) | ((uint64_t)__popcll(sn) << 32) |
                            ((uint64_t)__popcll(en) << 48);
        // (four 16-bit counts, totals <= 4096: the halves scan apart)
        const uint32_t ci_lo = wave_incl_add_dpp((uint32_t)cc), ci_hi = wave_incl_add_dpp((uint32_t)(cc >> 32));
        const uint64_t ci = (uint64_t)ci_lo | ((uint64_t)ci_hi << 32);
        const uint64_t ct = (uint64_t)lane_val(ci_lo, 63) | ((uint64_t)lane_val(ci_hi, 63) << 32);
        const uint64_t cx = ci - cc;
        const int fl = hm ? first_lane(hm) : 0, ll = hm ? 63 - __builtin_clzll(hm) : 0;
        const uint32_t tf = (uint32_t)__shfl((int)first2, fl, 64), tl = (uint32_t)__shfl((int)last2, ll, 64);
        if (lane == 0) {
            rsl.rc[tile] = ct;
            rsl.rf[tile] = (hm ? 1 : 0) | (int32_t)(tf << 1) | (int32_t)(tl << 3);
        }
        if ((sl | el | sn | en) != 0) {   // (rare: a lane holds ~0.1 run boundaries)
            const int64_t o0 = toff[tile] + (int64_t)(ex & 0xffff);
            int32_t* const dst[4] = {rsl.sl, rsl.el, rsl.sn, rsl.en};
            const uint64_t ev[4] = {sl, el, sn, en};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t at = (uint32_t)(cx >> (16 * q)) & 0xffffu;
                for (uint64_t m = ev[q]; m; m &= m - 1) {
                    const int b = __builtin_ctzll(m);
                    if (at < RUN_SLOT) dst[q][(size_t)tile * RUN_SLOT + at] = (int32_t)(o0 + __popcll(keep & below64(b)));
                    else atomicOr(rsl.ovf, 1);
                    at++;
                }
            }
        }
    }
    if (flags && __ballot((keep & r.par) != 0) && lane == 0) atomicOr(flags, 1);
    if (out) {   // (null: only the filtered copy is wanted -- the reconstruction needs R' alone)
        stage_lane<false>(s1, tab, w, keep, (int)(ex & 0xffff));
        wave_sync();
        stage_out(st4, (int)(tot & 0xffff), out, toff[tile]);
    }
    if (out2) {
        if (out && !__ballot(fkeep != keep)) {   // the filter dropped nothing here: same bytes, uppercased
            stage_out<true>(st4, (int)(tot >> 16), out2, toff2[tile]);
        } else {
            wave_sync();
            stage_lane<true>(s1, tab, w, fkeep, (int)(ex >> 16));
            wave_sync();
            stage_out(st4, (int)(tot >> 16), out2, toff2[tile]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Stripped bytes on demand (round 6).  A pair whose mode the switch probe decides (local.hip
// k_local_probe) never reads the unfiltered stripped copies T and R unless it stays local, so the
// strips skip writing them (out = null) and the probe's 128 segments of each are materialised here
// from the FASTA and the write pass's tile offsets: the wave of slot i finds the tile holding
// stripped byte q0 = seg * SEG_L (the last tile whose output offset is <= q0), re-classifies that
// tile and the next ones exactly as k_strip_write does, and drops each kept byte that falls in
// [q0, q0 + SEG_L) into dst[i * SEG_B + (pos - q0)].  seg < 0: nothing (the slot stays unused).
// ---------------------------------------------------------------------------------------------
template <IngestMode MODE>
__global__ __launch_bounds__(64) void k_strip_gather(const uint8_t* __restrict__ buf, int64_t n,
                                                     const int64_t* __restrict__ hdr, const int64_t* __restrict__ toff,
                                                     const int32_t* __restrict__ tcarry, const int64_t* __restrict__ d_len,
                                                     const int32_t* __restrict__ segs, uint8_t* __restrict__ dst) {
    __shared__ uint4 tin[STRIP_WTILE / 16];
    const int lane = lane_id();
    const int32_t seg = segs[blockIdx.x];
    if (seg < 0) return;
    const int64_t len = *d_len;
    const int64_t q0 = (int64_t)seg * SEG_L;
    const int64_t q1 = q0 + SEG_L < len ? q0 + SEG_L : len;
    uint8_t* out = dst + (size_t)blockIdx.x * SEG_GATHER_B;
    if (q0 >= q1) return;
    const int64_t ntiles = (n + STRIP_WTILE - 1) / STRIP_WTILE;
    // last tile t with toff[t] <= q0 (toff is nondecreasing; toff[0] = 0): a 64-way search, one
    // probe per lane and step (three dependent round trips for a chr1-sized FASTA, not sixteen)
    int64_t lo = 0, hi = ntiles - 1;   // invariant: toff[lo] <= q0, the answer is in [lo, hi]
    while (lo < hi) {
        const int64_t span = hi - lo;
        const int64_t p = lo + (span * (lane + 1) + 63) / 64;   // lane 63 probes hi
        const bool le = p <= hi && toff[p] <= q0;
        const unsigned long long m = __ballot(le);
        if (!m) { hi = lo + (span + 63) / 64 - 1; if (hi < lo) hi = lo; continue; }
        const int l = 63 - __builtin_clzll(m);
        const int64_t pl = lo + (span * (l + 1) + 63) / 64;
        const int64_t pn = l < 63 ? lo + (span * (l + 2) + 63) / 64 - 1 : hi;
        lo = pl;
        hi = pn < hi ? pn : hi;
        if (hi < lo) hi = lo;
    }
    const int64_t h = MODE == INGEST_TGT ? hdr[0] : 0, he = MODE == INGEST_TGT ? hdr[1] : 0;
    for (int64_t tile = lo; tile < ntiles && toff[tile] < q1; tile++) {
        const int64_t off = tile * STRIP_WTILE + (int64_t)lane * SL;
        uint32_t w[SNW];
        int32_t prior;
        uint64_t lsm;
        const StripMasks r = strip_tile<MODE>(FILTER_UPPER, buf, n, h, he, off, w, prior, lsm, tin);
        int32_t pr = prior;
        if (MODE == INGEST_REF && pr < 0) pr = tcarry[tile];
        const uint64_t keep = r.known | (pr == 1 ? r.unknown : 0ull);
        const uint32_t c = (uint32_t)__popcll(keep);
        const uint32_t ex = wave_incl_add<uint32_t>(c) - c;
        int64_t pos = toff[tile] + ex;
        if (pos < q1 && pos + c > q0) {
            for (uint64_t m = keep; m; m &= m - 1, pos++) {
                const int b = __builtin_ctzll(m);
                if (pos >= q0 && pos < q1) out[pos - q0] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
            }
        }
        wave_sync();   // (tin is reused by the next tile)
    }
}

// ---------------------------------------------------------------------------------------------
// runs of a predicate
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool run_pred(RunPred p, uint8_t c) {
    return p == RUN_LOWER ? c_islower(c) : (c == 'N' || c == 'n');
}

// bit i: pred(byte off + i) for both predicates (SWAR); bytes past n are not in any run
__device__ __forceinline__ void pred_masks(const uint8_t* __restrict__ in, int64_t n, int64_t off, uint32_t& ml,
                                           uint32_t& mn) {
    uint32_t w[PER_T / 4];
    load_words(in, n, off, w);   // pads with ' ' (in no run)
    ml = 0;
    mn = 0;
#pragma unroll
    for (int q = 0; q < PER_T / 4; q++) {
        const uint32_t x = w[q];
        ml |= sw_bits(sw_lt(x, 'z' + 1) & ~sw_lt(x, 'a')) << (4 * q);
        mn |= sw_bits(sw_eq(x, 'N') | sw_eq(x, 'n')) << (4 * q);
    }
}

// Both run lines' predicates in one pass (counts of two predicates packed in one 32-bit block
// scan: a tile holds at most 4096 runs of each).
__global__ __launch_bounds__(SCCG_BLOCK) void k_runs_count(const uint8_t* __restrict__ in, int64_t n,
                                                           int64_t* __restrict__ cnt_l, int64_t* __restrict__ cnt_n) {
    __shared__ int32_t tmp32[8];
    const int64_t off = (int64_t)blockIdx.x * INGEST_TILE + (int64_t)threadIdx.x * PER_T;
    uint32_t ml, mn;
    pred_masks(in, n, off, ml, mn);
    const bool in_prev = off > 0 && off - 1 < n;
    const uint32_t pl = in_prev && run_pred(RUN_LOWER, in[off - 1]), pn = in_prev && run_pred(RUN_N, in[off - 1]);
    const int32_t c = __popc(ml & ~((ml << 1) | pl)) | (__popc(mn & ~((mn << 1) | pn)) << 16);
    int32_t tot;
    block_excl_add<int32_t>(c, tmp32, &tot);
    if (threadIdx.x == 0) { cnt_l[blockIdx.x] = tot & 0xffff; cnt_n[blockIdx.x] = tot >> 16; }
}

__device__ __forceinline__ void put_positions(uint32_t bits, int64_t off, int32_t* __restrict__ dst, int64_t at) {
    while (bits) {
        dst[at++] = (int32_t)(off + __ffs((int)bits) - 1);
        bits &= bits - 1;
    }
}

__global__ __launch_bounds__(SCCG_BLOCK) void k_runs_write(const uint8_t* __restrict__ in, int64_t n,
                                                           const int64_t* __restrict__ toff_l,
                                                           const int64_t* __restrict__ toff_n, int32_t* __restrict__ rs_l,
                                                           int32_t* __restrict__ re_l, int32_t* __restrict__ rs_n,
                                                           int32_t* __restrict__ re_n) {
    __shared__ int32_t tmp32[8];
    const int64_t tile0 = (int64_t)blockIdx.x * INGEST_TILE;
    const int64_t off = tile0 + (int64_t)threadIdx.x * PER_T;
    uint32_t ml, mn;
    pred_masks(in, n, off, ml, mn);
    const bool in_prev = off > 0 && off - 1 < n, in_next = off + PER_T < n;
    const uint32_t pl = in_prev && run_pred(RUN_LOWER, in[off - 1]), pn = in_prev && run_pred(RUN_N, in[off - 1]);
    const uint32_t nl = in_next && run_pred(RUN_LOWER, in[off + PER_T]), nn = in_next && run_pred(RUN_N, in[off + PER_T]);
    const uint32_t sl = ml & ~((ml << 1) | pl), el = ml & ~((ml >> 1) | (nl << 31));
    const uint32_t sn = mn & ~((mn << 1) | pn), en = mn & ~((mn >> 1) | (nn << 31));
    // runs open across the tile start end inside this tile (or later) but started before it
    const bool t_in = tile0 > 0 && tile0 < n;
    const bool open_l = t_in && run_pred(RUN_LOWER, in[tile0 - 1]) && run_pred(RUN_LOWER, in[tile0]);
    const bool open_n = t_in && run_pred(RUN_N, in[tile0 - 1]) && run_pred(RUN_N, in[tile0]);
    const int32_t xs = block_excl_add<int32_t>(__popc(sl) | (__popc(sn) << 16), tmp32, nullptr);
    const int32_t xe = block_excl_add<int32_t>(__popc(el) | (__popc(en) << 16), tmp32, nullptr);
    put_positions(sl, off, rs_l, toff_l[blockIdx.x] + (xs & 0xffff));
    put_positions(el, off, re_l, toff_l[blockIdx.x] - (open_l ? 1 : 0) + (xe & 0xffff));
    put_positions(sn, off, rs_n, toff_n[blockIdx.x] + (xs >> 16));
    put_positions(en, off, re_n, toff_n[blockIdx.x] - (open_n ? 1 : 0) + (xe >> 16));
}

// ---- the run arrays from the target strip's per-tile event slots (RUNS)
// per tile: its event counts plus the tile-boundary event (its first kept byte against the previous
// kept byte: the last kept byte of the nearest earlier tile that has one; none at the stream start)
constexpr int RUNS_LOOKBACK = 64;   // tiles without a kept byte crossed looking for it (more: ovf, fallback)
__global__ void k_runs_tiles(int64_t ntiles, const uint64_t* __restrict__ rc, const int32_t* __restrict__ rf,
                             int64_t* __restrict__ cs, int64_t* __restrict__ ce, int32_t* __restrict__ bev,
                             int32_t* __restrict__ ovf) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t f = rf[t];
        const uint64_t c = rc[t];
        int32_t b = 0;
        if (f & 1) {
            uint32_t prev = 0;
            int64_t q = t - 1;
            for (; q >= 0 && t - q <= RUNS_LOOKBACK; q--) {
                const int32_t g = rf[q];
                if (g & 1) { prev = (uint32_t)(g >> 3) & 3u; break; }
            }
            if (q >= 0 && t - q > RUNS_LOOKBACK) atomicOr(ovf, 2);
            const uint32_t first = (uint32_t)(f >> 1) & 3u;
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const uint32_t fp = (first >> p) & 1u, pp = (prev >> p) & 1u;
                if (fp && !pp) b |= 1 << (2 * p);
                if (!fp && pp) b |= 2 << (2 * p);
            }
        }
        bev[t] = b;
        cs[t] = (int64_t)((c & 0xffff) + (b & 1)) | ((int64_t)(((c >> 32) & 0xffff) + ((b >> 2) & 1)) << 32);
        ce[t] = (int64_t)(((c >> 16) & 0xffff) + ((b >> 1) & 1)) | ((int64_t)((c >> 48) + ((b >> 3) & 1)) << 32);
    }
}

// per tile: its boundary event, then its slot events, at the scanned offsets (ends inclusive)
__global__ void k_runs_copy(int64_t ntiles, const int64_t* __restrict__ toff, const uint64_t* __restrict__ rc,
                            const int32_t* __restrict__ bev, const int64_t* __restrict__ cs, const int64_t* __restrict__ ce,
                            RunSlots rsl, int32_t* __restrict__ rs_l, int32_t* __restrict__ re_l,
                            int32_t* __restrict__ rs_n, int32_t* __restrict__ re_n) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t c = rc[t];
        const int32_t b = bev[t];
        const int32_t t0 = (int32_t)toff[t];
        const size_t sb = (size_t)t * RUN_SLOT;
        int32_t* const dst[4] = {rs_l, re_l, rs_n, re_n};
        const int32_t* const src[4] = {rsl.sl, rsl.el, rsl.sn, rsl.en};
        const int64_t base[4] = {cs[t] & 0xffffffff, ce[t] & 0xffffffff, cs[t] >> 32, ce[t] >> 32};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int end = q & 1;   // ends are stored inclusive: the exclusive end - 1
            int64_t at = base[q];
            if ((b >> q) & 1) dst[q][at++] = t0 - end;
            const int nq = (int)((c >> (16 * q)) & 0xffff);
            for (int k = 0; k < nq && k < RUN_SLOT; k++) dst[q][at++] = src[q][sb + k] - end;
        }
    }
}

// counts; a run still open at the end ends at |T| - 1
__global__ void k_runs_fin(const int64_t* __restrict__ tot, const int64_t* __restrict__ d_nT, int32_t* __restrict__ re_l,
                           int32_t* __restrict__ re_n, int64_t* __restrict__ d_nruns) {
    const int64_t sl = tot[0] & 0xffffffff, sn = tot[0] >> 32, el = tot[1] & 0xffffffff, en = tot[1] >> 32;
    if (sl > el) re_l[sl - 1] = (int32_t)(*d_nT - 1);
    if (sn > en) re_n[sn - 1] = (int32_t)(*d_nT - 1);
    d_nruns[0] = sl;
    d_nruns[1] = sn;
}

// text of one run: "d," | "(d,len)" | final singleton "d" (compression.cpp:351-366)
__device__ __forceinline__ int64_t run_text_len(int32_t d, int32_t len, bool at_end) {
    return len == 1 ? (int64_t)ndigits_i32(d) + (at_end ? 0 : 1) : (int64_t)(3 + ndigits_i32(d) + ndigits_i32(len));
}

__global__ void k_run_textlen(const int32_t* __restrict__ rs, const int32_t* __restrict__ re, int64_t nr,
                              int64_t n, int64_t* __restrict__ len) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
        const int32_t d = rs[r] - (r ? rs[r - 1] : 0);
        len[r] = run_text_len(d, re[r] - rs[r] + 1, (int64_t)re[r] == n - 1);
    }
}

__global__ void k_run_textwrite(const int32_t* __restrict__ rs, const int32_t* __restrict__ re, int64_t nr,
                                int64_t n, const int64_t* __restrict__ off, uint8_t* __restrict__ out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
        const int32_t d = rs[r] - (r ? rs[r - 1] : 0);
        const int32_t len = re[r] - rs[r] + 1;
        uint8_t* o = out + off[r];
        if (len == 1) {
            o += write_i32(o, d);
            if ((int64_t)re[r] != n - 1) *o = ',';
        } else {
            *o++ = '(';
            o += write_i32(o, d);
            *o++ = ',';
            o += write_i32(o, len);
            *o = ')';
        }
    }
}

}  // namespace

// The target's header in one single-block launch: the first '>' at a line start, then the first
// '\n' after it, 16 KiB per block step (a FASTA header sits at byte 0, so this is one or two steps;
// a target without one is scanned to its end by this block, ~1 us per 16 KiB).  It replaces an
// init launch and two 64-block ticket searches, which in multi-context runs waited ~50 us each for
// CU slots behind the other context's grids.  d_sc[0] = header start (n: none), d_sc[1] = its '\n'
// (n: none), d_sc[2..3] = 0.
constexpr int FH_T = 256, FH_PER = 64;   // (a 1024-thread block would wait for a whole free CU)
__global__ __launch_bounds__(FH_T) void k_find_header(const uint8_t* __restrict__ buf, int64_t n, int64_t* __restrict__ d_sc) {
    __shared__ unsigned long long s_hit;
    int64_t res[2] = {n, n};
    for (int ph = 0; ph < 2; ph++) {
        if (ph == 1 && res[0] >= n) break;
        const int64_t from = ph == 0 ? 0 : res[0] + 1;
        for (int64_t cs = from & ~(int64_t)63; cs < n; cs += (int64_t)FH_T * FH_PER) {
            if (threadIdx.x == 0) s_hit = ~0ull;
            __syncthreads();
            const int64_t p0 = cs + (int64_t)threadIdx.x * FH_PER;
            if (p0 < n) {
                uint32_t w[FH_PER / 4];
                load_words<FH_PER / 4>(buf, n, p0, w);
                uint8_t prev = p0 > 0 ? buf[p0 - 1] : (uint8_t)'\n';
                int64_t hit = -1;
#pragma unroll
                for (int i = 0; i < FH_PER; i++) {
                    const uint8_t c = wb(w, i);
                    const int64_t p = p0 + i;
                    const bool ok = p >= from && p < n && (ph == 0 ? (c == '>' && prev == '\n') : c == '\n');
                    if (ok && hit < 0) hit = p;
                    prev = c;
                }
                if (hit >= 0) atomicMin(&s_hit, (unsigned long long)hit);
            }
            __syncthreads();
            const unsigned long long h = s_hit;
            __syncthreads();   // (s_hit is reset next step)
            if (h != ~0ull) { res[ph] = (int64_t)h; break; }
        }
    }
    if (threadIdx.x == 0) { d_sc[0] = res[0]; d_sc[1] = res[1]; d_sc[2] = 0; d_sc[3] = 0; }
}

// =============================================================================================
int launch_first_match(const uint8_t* buf, int64_t n, const int64_t* from_slot, int mode, uint8_t c, int64_t* res,
                       int64_t* ticket_slot, hipStream_t s) {
    int rc = dev_set_i64(res, 1, {n}, s);
    if (!rc) rc = dev_set_i64(ticket_slot, 1, {0}, s);
    if (rc) return rc;
    if (n > 0) {
        hipLaunchKernelGGL(k_first_match, dim3(64), dim3(SCCG_BLOCK), 0, s, buf, n, from_slot, mode, c, res,
                           reinterpret_cast<unsigned int*>(ticket_slot));
        SCCG_HIP(hipGetLastError());
    }
    return 0;
}

int launch_find_header(const uint8_t* buf, int64_t n, int64_t* d_sc, hipStream_t s) {
    // d_sc[0] = header start (first '>' at a line start), d_sc[1] = its '\n' (n if none);
    // d_sc[2], d_sc[3] are the chunk tickets (free for the caller afterwards); one init launch
    hipLaunchKernelGGL(k_find_header, dim3(1), dim3(FH_T), 0, s, buf, n, d_sc);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_fasta_strip(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header, uint8_t* out,
                       int64_t* d_len, int32_t* d_flags, const IngestScratch& sc, hipStream_t s, FilterMode fmode,
                       uint8_t* out2, int64_t* d_len2, const RunSlots* runs) {
    if (n <= 0) {
        SCCG_HIP(hipMemsetAsync(d_len, 0, sizeof(int64_t), s));
        if (d_len2) SCCG_HIP(hipMemsetAsync(d_len2, 0, sizeof(int64_t), s));
        return 0;
    }
    if (!out2) fmode = FILTER_UPPER;   // second output unused
    const int64_t ntiles = (n + STRIP_TILE - 1) / STRIP_TILE;
    const unsigned g = grid_for(ntiles, WPB);
    uint16_t* const kc = sc.keep_cache;
    int32_t* const kf = sc.keep_flag;
#define SUMMARY(M, K)                                                                                                   \
    hipLaunchKernelGGL((k_strip_summary<M, K>), dim3(g), dim3(SCCG_BLOCK), 0, s, fmode, buf, n, d_header, sc.tile_a,   \
                       sc.tile_b, sc.tile_fa, sc.tile_fb, sc.tile_last, kc, kf)
    if (mode == INGEST_TGT && kc) SUMMARY(INGEST_TGT, true);
    else if (mode == INGEST_TGT) SUMMARY(INGEST_TGT, false);
    else if (kc) SUMMARY(INGEST_REF, true);
    else SUMMARY(INGEST_REF, false);
#undef SUMMARY
    const int64_t nblk = (ntiles + SCAN_B - 1) / SCAN_B;
    if (nblk > SCAN_B) return SCCG_E_UNSUPPORTED;   // > 4 GiB of FASTA
    TileSum* btot = reinterpret_cast<TileSum*>(sc.block_sums);
    hipLaunchKernelGGL(k_strip_scan_local, dim3((unsigned)nblk), dim3(SCAN_T), 0, s, ntiles, sc.tile_a, sc.tile_b,
                       sc.tile_fa, sc.tile_fb, sc.tile_last, btot);
    hipLaunchKernelGGL(k_strip_scan_blocks, dim3(1), dim3(SCAN_T), 0, s, nblk, btot);
    hipLaunchKernelGGL(k_strip_scan_apply, dim3(grid_for(ntiles, 256)), dim3(256), 0, s, ntiles, sc.tile_a, sc.tile_b,
                       sc.tile_fa, sc.tile_fb, sc.tile_last, btot, sc.tile_off, sc.tile_off2, sc.tile_carry, d_len,
                       d_len2);
    const RunSlots rsl = runs ? *runs : RunSlots{};
    if (mode == INGEST_TGT && runs)
        PROF_LAUNCH(PROF_STRIP, s, (k_strip_write<INGEST_TGT, true>), dim3(g), dim3(SCCG_BLOCK), 0, s, fmode, buf, n, d_header,
                    sc.tile_off, sc.tile_off2, sc.tile_carry, out, out2, d_flags, rsl, (const uint16_t*)kc, (const int32_t*)kf);
    else if (mode == INGEST_TGT)
        PROF_LAUNCH(PROF_STRIP, s, (k_strip_write<INGEST_TGT, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, fmode, buf, n, d_header,
                    sc.tile_off, sc.tile_off2, sc.tile_carry, out, out2, d_flags, rsl, (const uint16_t*)kc, (const int32_t*)kf);
    else
        PROF_LAUNCH(PROF_STRIP, s, (k_strip_write<INGEST_REF, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, fmode, buf, n, d_header,
                    sc.tile_off, sc.tile_off2, sc.tile_carry, out, out2, d_flags, rsl, (const uint16_t*)kc, (const int32_t*)kf);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_runs2(const uint8_t* in, int64_t n, int32_t* rs_l, int32_t* re_l, int32_t* rs_n, int32_t* re_n,
                 int64_t* d_nruns, int64_t* d_cnt_l, int64_t* d_cnt_n, int64_t* d_partial, hipStream_t s) {
    if (n <= 0) {
        SCCG_HIP(hipMemsetAsync(d_nruns, 0, 2 * sizeof(int64_t), s));
        return 0;
    }
    const int64_t ntiles = (n + INGEST_TILE - 1) / INGEST_TILE;
    hipLaunchKernelGGL(k_runs_count, dim3((unsigned)ntiles), dim3(SCCG_BLOCK), 0, s, in, n, d_cnt_l, d_cnt_n);
    int rc = dev_excl_sum(d_cnt_l, d_cnt_l, ntiles, d_nruns, d_partial, s);
    if (!rc) rc = dev_excl_sum(d_cnt_n, d_cnt_n, ntiles, d_nruns + 1, d_partial, s);
    if (rc) return rc;
    PROF_LAUNCH(PROF_RUNS, s, k_runs_write, dim3((unsigned)ntiles), dim3(SCCG_BLOCK), 0, s, in, n,
                (const int64_t*)d_cnt_l, (const int64_t*)d_cnt_n, rs_l, re_l, rs_n, re_n);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_runs_from_strip(const RunSlots& rs, int64_t ntiles, const int64_t* toff, const int64_t* d_nT, int32_t* rs_l,
                           int32_t* re_l, int32_t* rs_n, int32_t* re_n, int64_t* d_nruns, int64_t* cs, int64_t* ce,
                           int32_t* bev, int64_t* d_tot, int64_t* d_partial, hipStream_t s) {
    const unsigned g = grid_for(ntiles, 256) > 4096 ? 4096 : grid_for(ntiles, 256);
    hipLaunchKernelGGL(k_runs_tiles, dim3(g), dim3(256), 0, s, ntiles, (const uint64_t*)rs.rc, (const int32_t*)rs.rf, cs, ce,
                       bev, rs.ovf);
    if (const int rc = dev_excl_sum2(cs, cs, d_tot, ce, ce, d_tot + 1, ntiles, d_partial, s)) return rc;
    PROF_LAUNCH(PROF_RUNS, s, k_runs_copy, dim3(g), dim3(256), 0, s, ntiles, toff, (const uint64_t*)rs.rc, (const int32_t*)bev,
                (const int64_t*)cs, (const int64_t*)ce, rs, rs_l, re_l, rs_n, re_n);
    hipLaunchKernelGGL(k_runs_fin, dim3(1), dim3(1), 0, s, (const int64_t*)d_tot, d_nT, re_l, re_n, d_nruns);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_run_text(const int32_t* rs, const int32_t* re, int64_t nruns, int64_t n, uint8_t* out, int64_t* d_len,
                    int64_t* d_tmp, int64_t* d_partial, hipStream_t s) {
    if (nruns <= 0) {
        SCCG_HIP(hipMemsetAsync(d_len, 0, sizeof(int64_t), s));
        return 0;
    }
    const unsigned g = grid_for(nruns, 256) > 4096 ? 4096 : grid_for(nruns, 256);
    hipLaunchKernelGGL(k_run_textlen, dim3(g), dim3(256), 0, s, rs, re, nruns, n, d_tmp);
    int rc = dev_excl_sum(d_tmp, d_tmp, nruns, d_len, d_partial, s);
    if (rc) return rc;
    PROF_LAUNCH(PROF_RUNTEXT, s, k_run_textwrite, dim3(g), dim3(256), 0, s, rs, re, nruns, n, (const int64_t*)d_tmp, out);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int launch_strip_gather(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header, const int64_t* toff,
                        const int32_t* tcarry, const int64_t* d_len, const int32_t* segs, int nslots, uint8_t* dst,
                        hipStream_t s) {
    if (n <= 0 || nslots <= 0) return 0;
    if (mode == INGEST_TGT)
        hipLaunchKernelGGL(k_strip_gather<INGEST_TGT>, dim3(nslots), dim3(64), 0, s, buf, n, d_header, toff, tcarry, d_len,
                           segs, dst);
    else
        hipLaunchKernelGGL(k_strip_gather<INGEST_REF>, dim3(nslots), dim3(64), 0, s, buf, n, d_header, toff, tcarry, d_len,
                           segs, dst);
    SCCG_HIP(hipGetLastError());
    return 0;
}

// the unfiltered stripped copy alone (out), from the tile offsets of an earlier launch_fasta_strip
// of the same input (its scan results are still in sc): the write pass again, without the filter
int launch_strip_rewrite(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header, uint8_t* out,
                         const IngestScratch& sc, hipStream_t s) {
    if (n <= 0) return 0;
    const int64_t ntiles = (n + STRIP_TILE - 1) / STRIP_TILE;
    const unsigned g = grid_for(ntiles, WPB);
    const RunSlots rsl{};
    if (mode == INGEST_TGT)
        PROF_LAUNCH(PROF_STRIP, s, (k_strip_write<INGEST_TGT, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, FILTER_UPPER, buf, n,
                    d_header, sc.tile_off, sc.tile_off2, sc.tile_carry, out, (uint8_t*)nullptr, (int32_t*)nullptr, rsl,
                    (const uint16_t*)nullptr, (const int32_t*)nullptr);
    else
        PROF_LAUNCH(PROF_STRIP, s, (k_strip_write<INGEST_REF, false>), dim3(g), dim3(SCCG_BLOCK), 0, s, FILTER_UPPER, buf, n,
                    d_header, sc.tile_off, sc.tile_off2, sc.tile_carry, out, (uint8_t*)nullptr, (int32_t*)nullptr, rsl,
                    (const uint16_t*)nullptr, (const int32_t*)nullptr);
    SCCG_HIP(hipGetLastError());
    return 0;
}
