// walk.hip -- global mode: match_sequences(R', T', 14, 100, true) and its record text.
//
//   compression.cpp:561  match_sequences(reference_genome, target_genome, k, m, true)
//   compression.cpp:64-161 greedy walk, :83-101 +-m range gate, :110-138 selection
//   compression.cpp:564-573 record emission, :222-304 delta_encode
//
// The walk is sequential through its state (index, prev_match_end = P).  Two observations make
// it parallel and exact:
//   1. Once P != -1 the gate admits only candidates c in [P-m, P+m]; a gated step is therefore a
//      function of the target k-mer and the 2m+k reference bytes around P, never of the full
//      k-mer table: an LDS-resident window of <= 201 keys decides both "literal" and the
//      candidate set (the ungated l1/p1 of :124-129 is only consulted when the gated pick is the
//      pn2==0 sentinel, i.e. p2 == 0, which needs P <= m -- handled by an exact full scan).
//   2. Two walks that reach the same (index, P) coincide from then on.  So the target is cut into
//      chunks; round 1 walks every chunk speculatively from a guessed P (a 32-mer anchor on a
//      1/16-sampled reference index); later rounds re-walk a chunk from its predecessor's exit
//      state until it emits a match its previous trajectory also holds (then the rest of the
//      trajectory is kept).  Rounds repeat until every chunk was walked from its true entry.
// The first step (P == -1, ungated) and the p2 == 0 escalations run as exact grid-wide scans.
#include "internal.h"

#include <algorithm>
#include <chrono>
#include <map>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

constexpr int WPB = 4;                 // chunks (waves) per block
// k_walk's waves per block (SCCG_WALK_WPB for A/B builds): a block's LDS is released only when all
// its waves are done, so fewer waves per block let the dispatcher start the next chunk sooner
#ifndef SCCG_WALK_WPB
#define SCCG_WALK_WPB 4
#endif
constexpr int WWPB = SCCG_WALK_WPB;
constexpr int WCAP = 256;              // window positions held in LDS (2m+1 <= WCAP)
constexpr int32_t INVALID = INT32_MIN;
constexpr int32_t NEVER = INT32_MIN + 1;   // usedX of a chunk never walked: differs from every state
constexpr int ANCHOR_K = 32;
// Walk keys are exact 2-bit codes of at most KEY_K bases (common.h).  For k > KEY_K (a non-parity
// parameter override; the reference hard-codes k = 14, compression.cpp:373) every key is the code of
// the k-mer's first KEY_K bases: a key hit is a candidate only if the extension from KEY_K reaches
// k (ext_k), and a position whose key hits have no such candidate is a literal step.
constexpr int KEY_K = 15;
constexpr int KMAX = 32;              // largest k the walk takes
constexpr int KB_COUNT = 32;          // kb: the first k bytes of T' at [0, k), their count at [32, 36)
// Reference sample stride (SCCG_ANCHOR_STEP for tuning runs).  Round 5: 64 instead of 32 -- half the
// table's scattered 8-byte writes (the early sweep's dominant cost: genome bench 4.0-4.4 -> 2.0 ms
// of sweep per step, gpurun_out/r05r) and no loss in the walk's speculation (hg genome walk and
// rounds unchanged; a 256-position vote window still holds ~4 samples of an aligned stretch).
constexpr int ANCHOR_STEP_DEFAULT = 64;
constexpr int ANCHOR_LOAD_DEFAULT = 1;    // table slots per sample, rounded up to a power of two (SCCG_ANCHOR_LOAD):
                                          // a 64 MiB table for chr1 stays in the MALL (4 slots/sample: 256 MiB, sweep +40 %)
#ifndef ANCHOR_PROBE_BATCHES
#define ANCHOR_PROBE_BATCHES 2            // 64 target probes per batch per anchor vote (measured: 2 beats 4)
#endif
constexpr uint32_t A_MULTI = 0xFFFFFFFFu;    // anchor position of a 32-mer seen more than once
constexpr int ANCHOR_RETRIES = 8;             // later votes for a chunk whose start has none
constexpr int32_t ANCHOR_RETRY_STEP = 512;    // target bases between them
constexpr int32_t FROZEN_MIN = 4096;   // literal bases at a chunk end that trigger a frozen-P scan
constexpr int FROZEN_MAX = 256;        // frozen chunks handled per batch (grid.y of k_frozen_scan)
constexpr int FROZEN_FIRST = 16;       // the batch launched blind, before the round's sync

enum ChunkKind : int32_t { KIND_SPEC = 0, KIND_FIX = 1, KIND_RESUME = 2 };
enum ChunkStatus : int32_t { ST_OK = 0, ST_ESC = 1, ST_CONV = 3, ST_DONE = 4, ST_TRUNC = 5 };
// A fix-up whose predecessor is re-walked in the same round starts from a stale entry: its result
// counts only if it converges, so it gives up after this many target positions without converging
// (a stale entry is often garbage, whose walk is a chunk-long stuck literal scan).
constexpr int32_t STALE_BUDGET_DEFAULT = 0;   // 0: off (SCCG_STALE_BUDGET sets it for tuning runs)
// A speculative walk that has gone RESEED_GAP target positions without a match re-seeds P from a
// fresh anchor vote at its position: a bad start guess otherwise leaves it stuck in a chunk-long
// literal scan.  The trajectory is then a walk from a different state after the re-seed, so a
// later fix-up may converge only onto its matches from the re-seed on (seedq).
constexpr int32_t RESEED_GAP = 1024;
// A fix-up that crossed at least half its chunk while P moved less than TRAP_P is "trapped": the
// sequential walk is stuck near one reference window (a frozen P, or chance hits inside a
// low-complexity window that keep nudging P).  Its successors are then usually trapped near the
// same P, so up to RESPEC_AHEAD chunks after the next pending one are walked again speculatively
// from that P in the same round, instead of resolving one chunk per round.
constexpr int32_t TRAP_P = 4096;
constexpr int RESPEC_AHEAD = 256;
constexpr int RESPEC_MAX_TRIGGERS = 64;
constexpr int32_t UNGUESSED_LOOKBACK = 64;   // chunks back k_round_pending looks for a diagonal
constexpr int32_t LONG_GAP = 4096;   // literal gaps of the record text copied grid-wide
constexpr int32_t CAND_CAP = 65536;  // early sweep: first-k-mer occurrences kept (more: full sweep later)
// Frozen chains (k_chain_*): a committed frozen chunk's exit state is walked on over the rest of the
// target by one wave that visits only "band hits" -- target positions whose k-mer occurs among the
// reference k-mers within CH_BAND of the generation's P -- found by a grid scan.
#ifndef SCCG_CH_BAND
#define SCCG_CH_BAND 512
#endif
constexpr int CH_BAND = SCCG_CH_BAND;   // band half-width (reference positions around P)
constexpr int CH_TBITS = CH_BAND <= 2048 ? 13 : 14;   // band key table: 8192 / 16384 LDS slots (load <= 1/2)
#ifndef SCCG_CH_GRID
#define SCCG_CH_GRID 512
#endif
constexpr int CH_GRID = SCCG_CH_GRID;  // scan blocks (1024 threads, 16 positions each per step)
constexpr int CH_HCAP = 4096;          // band hits kept per block and generation
constexpr int32_t CHAIN_MCAP = 1 << 22;   // matches a chain may take
#ifndef SCCG_CH_GENS_PER_SYNC
#define SCCG_CH_GENS_PER_SYNC 4
#endif
constexpr int CH_GENS_PER_SYNC = SCCG_CH_GENS_PER_SYNC;    // generations queued per host check
constexpr int ROUND_BATCH_DEFAULT = 1;   // rounds queued per host readback from ROUND_BATCH_FROM on (1: off; A/B pending)
constexpr int ROUND_BATCH_FROM = 4;
constexpr int FF_MIN_CHUNKS = 8;       // frozen-first start: chunk 0's walk stuck for at least this many chunks
// SCCG_RECHUNK=1 (opt-in): a frozen-first (stuck, literal-heavy: T2T-like) target is walked again
// in chunks of FF_CHUNK bases.  Its divergent stretches hold ~400 short matches per 16 Ki chunk,
// each a latency-bound walk step, so the round's slowest chunks set the walk: the 100 Mb T2T-like
// pair 10.4 -> 8.3 ms and 20 Mb pairs -20..-30 %.  But on the T2T-like whole genome (24 pairs at
// UCSC lengths) the smaller chunks multiply the poorly-speculated ones that the rounds resolve one
// by one: chr3 44 -> 231 ms (72 -> 323 rounds), chr6 33 -> 186 ms, genome 0.50 -> 0.86 s
// (profiles/r03/rechunk_ab/) -- so the default keeps the size rule.
constexpr int FF_CHUNK = 8192;
#ifndef SCCG_CH_FF_SPAN
#define SCCG_CH_FF_SPAN (32 * 1024)
#endif
// find-first generations scan at most CH_GRID * CH_FF_SPAN target positions (then the next one goes
// on from there): a scan over the whole rest of the target kept every block before the hit busy
// for its whole span (T2T-like 100 Mb pair: ~73 us per generation, 40 generations)
constexpr int64_t CH_FF_SPAN = SCCG_CH_FF_SPAN;
constexpr int CH_MAX_GENS = 4096;      // generations per chain
constexpr int MARCH_ROUNDS = 4;        // rounds settling <= 2 chunks each before a march chain
constexpr int64_t CH_DENSE_HITS = 32768;  // band hits of one generation that switch the chain to find-first generations
constexpr int CH_DENSE_N = 32;         // hand back to the chunk rounds when CH_DENSE_N matches
constexpr int32_t CH_DENSE_SPAN = 8192;   // fall within this many target bases (the walk is aligned again)
// A chain is for frozen stretches (a chance hit every ~100 kb: T2T-like targets).  One that keeps
// finding matches is a trapped walk (chance hits in a low-complexity window nudging P every few kb,
// e.g. the synthetic chr22 from 45.8 Mb): one wave then walks them serially (~4 us each), which the
// rounds' trapped re-speculation resolves faster, so the chain hands back after this many matches.
#ifndef SCCG_CH_HANDBACK
#define SCCG_CH_HANDBACK 64
#endif
constexpr int CH_HANDBACK_N = SCCG_CH_HANDBACK;

struct WalkPtrs {
    const uint8_t* R;
    const uint8_t* T;
    int32_t nR, nT, k, m, S, C, cap;
    int32_t kp;               // key length: min(k, KEY_K); k > KEY_K confirms the rest by extension (KEY_K)
    // the target range the chunks cover: [xlo, xhi) (the whole T' = [0, nT) except for a range walk,
    // sccg_walk_range: the walk from a given state stops at the first index >= xhi)
    int32_t xlo, xhi;
    int32_t* bt[2];
    int32_t* bp[2];
    int32_t* bl[2];
    int32_t* cnt[2];
    int32_t* cur;
    int32_t* exitX;
    int32_t* exitP;
    int32_t* usedX;
    int32_t* usedP;
    int32_t* kind;
    int32_t* status;
    int32_t* escX;
    int32_t* escP;
    int32_t* escN;
    int32_t* escQ;
    int32_t* snapX;
    int32_t* snapP;
    int32_t* guess;
    int32_t* plist;       // chunks walked in the current round
    int32_t* rlist;       // chunks resumed after an escalation
    int32_t* clist;       // chunks a fix-up carries on into (k_walk<.., true>), count in scal[11]
    int32_t* newX;        // staged fix-up results (k_commit)
    int32_t* newP;
    int32_t* conv;
    int32_t* changed;
    int32_t* walked;      // round in which the chunk was last re-walked
    int32_t* lround;      // round for which the chunk was last put on the walk list
    int32_t* seedq;       // first match of the committed trajectory after its last re-seed
    int32_t* trapped;     // last fix-up walk (or frozen fill) of the chunk was trapped (TRAP_P)
    int32_t stale_budget; // positions a stale-entry fix-up may walk without converging (0: no limit)
    int32_t* frozen;      // fix-up ended in a long literal run at the chunk end
    int32_t* flist;       // committed frozen chunks of the round
    int32_t* fy;          // per listed frozen chunk: first window hit after its exit (k_frozen_scan)
    int32_t* scal;        // [0] pending count, [1] escalation count, [2] startX, [3] startP, [4] round,
                          // [5] frozen count, [6] frozen-scan first hit, [9] void round, [11] carry count,
                          // [12] trapped triggers of the round end, [13] frozen fills of the round end
    int32_t* trig;        // the round end's trapped triggers (RESPEC_MAX_TRIGGERS)
    int32_t* tflag;       // per chunk: round in which it was a trapped trigger (k_round_pending)
    int32_t unguessed_spec;   // SCCG_UNGUESSED_SPEC: k_round_pending speculates chunks left without a trajectory
    int32_t* fa_j;        // the round end's frozen fills: chunks fa_j+1 .. fa_l literal with P fa_p (scal[13])
    int32_t* fa_l;
    int32_t* fa_p;
    int32_t* hintY;       // per chunk: a frozen scan's first window hit of P = hintP in this chunk (-1: none);
    int32_t* hintP;       // a walk at (x <= hintY, hintP) in the chunk may jump to hintY (all literal steps)
    int32_t skip_hints;   // SCCG_SKIP_HINTS (default on)
    uint64_t* atab;
    uint32_t agen;            // anchor tag generation (one per call)
    int32_t adet;             // anchor slots written with atomicMax (SCCG_ANCHOR_DET, default off)
    uint32_t* fbits;          // the round's frozen / carry lists as chunk bitmaps (k_list_sort puts the
    uint32_t* cbits;          //   lists into chunk order from them and clears them)
    int32_t round;            // walk round of the launch (kernel argument copy)
    int32_t abits;
    const int64_t* dnR;       // early sweep: |R'| in device memory (nR is then only a bound)
    int32_t astep;            // anchor sample stride
    int32_t amulti;           // 1: second build pass marks repeated 32-mers
    unsigned long long* fc;   // full-candidate scan scalars: [0] lmax [1] cnt [2] has0 [3] minkey [4] firsthit [5] firstexo
                              // [8..11] the same four for the batch's first position (k_presence + k_cand_reduce)
    unsigned long long* fcb;  // per presence block: 4 candidate statistics
    int32_t* cand;            // early sweep: reference positions of the target's first k-mer (fc[13] of them)
    uint8_t* kb;              // early sweep: the target's first k bytes of T', read from its FASTA
    int64_t* flat_off;        // per chunk
    int32_t* ft;
    int32_t* fp;
    int32_t* fl;
    int64_t* tlen;            // per flat match: text length -> offsets
    int64_t* partial;
    int64_t* scal64;          // [0] total matches [1] text bytes [2] long literal gaps
    int64_t* lgap;            // long literal gaps of the record text: (source, destination, length) triples
    int64_t* cprev;           // per chunk: last earlier chunk holding a match (max-scan), then text offsets
    int64_t* ctext;           // per chunk: record text bytes of its target range -> offsets
    int64_t lgap_cap;
    // frozen chains (k_chain_*): state, the chain's matches, per-block band hits of a generation
    int32_t* chs;             // [0] active [1] x [2] P [3] matches [4] start chunk [5] end reason
                              // [6] band lo [7] band hi [8] generations [9] start x [10] start P
                              // [11] consecutive generations whose first block overflowed
                              // [12] mode (0 band hits, 1 find-first on the window) [13] first hit (mode 1)
    int32_t* chm_t;
    int32_t* chm_p;
    int32_t* chm_l;
    int32_t chm_cap;
    int32_t ch_settled;       // this chain starts only from a settled frozen chunk (march chains, host-set)
    int32_t* chh_y;           // CH_GRID x CH_HCAP band hits (position, key), in position order per block
    uint32_t* chh_k;
    int32_t* chh_n;           // per block: hits recorded, first position not covered (INT32_MAX: none)
    int32_t* chh_tr;
    uint64_t* dbg;            // SCCG_DEBUG: per chunk DBG_SLOTS counters (k_walk<K, true>)
    int32_t dbg_phases;       // SCCG_DEBUG_PHASES: also per-phase clocks
    int32_t dbg_round;        // SCCG_DEBUG_ROUND: keep the per-chunk counters of that round only (-1: the last)
};

// chunk j's target range [lo, hi)
__device__ __forceinline__ int32_t chunk_lo(const WalkPtrs& A, int32_t j) { return A.xlo + j * A.S; }
__device__ __forceinline__ int32_t chunk_hi(const WalkPtrs& A, int32_t j) {
    const int32_t lo = A.xlo + j * A.S;
    return lo + A.S < A.xhi ? lo + A.S : A.xhi;
}

// Per-wave LDS: the window's Bloom filter (wide literal scans) and a copy of the last 2 KiB the
// extension loaded from R' and from T'.  A match step reads its next window (R' around the new P),
// its next probe (T' right after the match) and usually the start of its next extension from that
// copy: after a match the walk continues on the same diagonal, inside the bytes it just compared.
// So most steps make no dependent HBM round trip at all; only an extension that runs past the copy
// loads (and refreshes it).
constexpr int WFBITS = 14;             // window pre-filter: 16384-bit Bloom filter, 3 hashes
#ifndef WALK_LBV
#define WALK_LBV 2048
#endif
constexpr int LBV = WALK_LBV;          // bytes of R' and of T' kept per wave (one HBM step loads them)
constexpr int LBW = LBV / 256;         // dwords of each per lane and HBM step
static_assert(LBW % 8 == 0, "whole 32-byte stretches per lane");
constexpr int LEAD = 128;              // of which before the extension's start (the next window reaches back m)
static_assert(LEAD % (4 * LBW) == 0, "the lead is whole lanes' stretches");
__device__ __forceinline__ uint32_t wf_h1(uint32_t key) { return slot_hash(key, WFBITS); }
__device__ __forceinline__ uint32_t wf_h2(uint32_t key) { return (key * 0x85EBCA77u) >> (32 - WFBITS); }
__device__ __forceinline__ uint32_t wf_h3(uint32_t key) { return (key * 0xC2B2AE3Du + 0x27D4EB2Fu) >> (32 - WFBITS); }
typedef __attribute__((address_space(1))) void GVoid;
typedef __attribute__((address_space(3))) void LVoid;
struct WalkLds {
    uint32_t wbits[1 << (WFBITS - 5)];
    __attribute__((aligned(16))) uint8_t rbuf[LBV + 64];   // R'[rb0, rb0 + LBV)  (+ slack read by the unaligned word loads)
    __attribute__((aligned(16))) uint8_t tbuf[LBV + 64];   // T'[tb0, tb0 + LBV)
};
// the copy's bases (wave-uniform); NO_BUF: nothing copied yet
constexpr int32_t NO_BUF = INT32_MIN / 2;
struct BufPos {
    int32_t rb0 = NO_BUF, tb0 = NO_BUF;
    __device__ __forceinline__ bool has_r(int32_t a, int32_t n) const { return a >= rb0 && a + n <= rb0 + LBV; }
    __device__ __forceinline__ bool has_t(int32_t a, int32_t n) const { return a >= tb0 && a + n <= tb0 + LBV; }
};

__device__ __forceinline__ uint64_t pick_key(int32_t p, int32_t pme) {
    const int32_t d = p - pme;
    return ((uint64_t)(uint32_t)(d < 0 ? -d : d) << 32) | (uint32_t)p;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, int k) {
    for (int i = 0; i < k; i++) if (a[i] != b[i]) return false;
    return true;
}

// ND words at byte offset off of an LDS byte array (ND + 1 aligned ds_read_b32)
template <int ND>
__device__ __forceinline__ void loadw_lds(const uint8_t* lds, int32_t off, uint32_t (&o)[ND]) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(lds) + (off >> 2);
    const uint32_t sh = (uint32_t)(off & 3);
    uint32_t v[ND + 1];
#pragma unroll
    for (int i = 0; i <= ND; i++) v[i] = w[i];
#pragma unroll
    for (int i = 0; i < ND; i++) o[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
}

// ND words at byte offset lds_off of an LDS copy (in_lds) or at g in global memory.  The empty asm
// after the global load keeps the compiler from merging the two loads into one FLAT load through a
// selected pointer (FLAT loads count against lgkmcnt: every later LDS wait would wait for HBM).
template <int ND>
__device__ __forceinline__ void loadw_sel(bool in_lds, const uint8_t* lds, int32_t lds_off, const uint8_t* g,
                                          uint32_t (&o)[ND]) {
    if (in_lds) {
        loadw_lds<ND>(lds, lds_off, o);
    } else {
        loadw<ND>(g, o);
        asm volatile("" ::: "memory");
    }
}

// first differing byte of two 4*N-byte stretches (4*N: none)
template <int N>
__device__ __forceinline__ int first_diff(const uint32_t (&r)[N], const uint32_t (&t)[N]) {
    int pos = 4 * N;
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
        const uint32_t x = r[i] ^ t[i];
        if (x) pos = 4 * i + (__builtin_ctz(x) >> 3);
    }
    return pos;
}
__device__ __forceinline__ int first_diff32(const uint32_t (&r)[8], const uint32_t (&t)[8]) { return first_diff<8>(r, t); }

// WALK_LCE_V (build option, A/B): 0 = lanes compare their own 32-byte stretches (the HBM step's
// loads compared straight from registers); 1 = coalesced 16-byte lanes through the LDS copy (the
// default since round 6: LDS bank-conflict cycles 65 -> 56 % of the LDS-active cycles, genome bench
// 151.6-162.1 -> 166.4-172.8 Gbase/s interleaved on one box, gpurun_out/r06n, profiles/r06/).
#ifndef WALK_LCE_V
#define WALK_LCE_V 1
#endif
#if WALK_LCE_V == 0
// longest common extension of R[a..] and T[b..], at most maxlen bytes (extend_alignment,
// compression.cpp:27-34); whole wave.  First from the LDS copy when both starts lie in it (2 KiB
// per pass); then from HBM, LBV bytes per round trip (lanes 0-3 load the LEAD bytes before the
// stretch compared), every HBM step leaving its bytes in the copy.
__device__ __forceinline__ int32_t wave_lce(const WalkPtrs& A, WalkLds& L, BufPos& B, int32_t a, int32_t b, int32_t maxlen) {
    const int lane = lane_id();
    if (maxlen <= 0) return 0;
    int32_t off = 0;
    if (a >= B.rb0 && b >= B.tb0 && a < B.rb0 + LBV && b < B.tb0 + LBV) {
        int32_t avail = B.rb0 + LBV - a < B.tb0 + LBV - b ? B.rb0 + LBV - a : B.tb0 + LBV - b;
        if (avail > maxlen) avail = maxlen;
        for (int32_t base = 0; base < avail; base += 2048) {
            const int32_t my = base + 32 * lane;
            int32_t e = INT32_MAX;
            if (my < avail) {
                uint32_t r[8], t[8];
                loadw_lds<8>(L.rbuf, a - B.rb0 + my, r);
                loadw_lds<8>(L.tbuf, b - B.tb0 + my, t);
                int pos = first_diff32(r, t);
                if (avail - my < 32 && pos >= avail - my) pos = avail - my == maxlen - my ? avail - my : 32;
                if (pos < 32) e = my + pos;
            }
            const unsigned long long sm = __ballot(e != INT32_MAX);
            if (sm) {
                const int32_t m = lane_val(e, first_lane(sm));
                return m < maxlen ? m : maxlen;
            }
        }
        if (avail >= maxlen) return maxlen;
        off = avail;
    }
    while (off < maxlen) {
        const int32_t lead = (a + off >= LEAD && b + off >= LEAD) ? LEAD : 0;
        const int32_t sa = a + off - lead, sb = b + off - lead;
        uint32_t r[LBW], t[LBW];
        loadw<LBW>(A.R + sa + 4 * LBW * lane, r);
        loadw<LBW>(A.T + sb + 4 * LBW * lane, t);
        wave_sync();   // the copy's previous readers are done
        {
            uint4* dr = reinterpret_cast<uint4*>(L.rbuf) + (LBW / 4) * lane;
            uint4* dt = reinterpret_cast<uint4*>(L.tbuf) + (LBW / 4) * lane;
#pragma unroll
            for (int i = 0; i < LBW / 4; i++) {
                dr[i] = make_uint4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
                dt[i] = make_uint4(t[4 * i], t[4 * i + 1], t[4 * i + 2], t[4 * i + 3]);
            }
        }
        wave_sync();
        B.rb0 = sa;
        B.tb0 = sb;
        const int32_t rel = 4 * LBW * lane - lead;   // this lane's bytes, from a + off
        int32_t e = INT32_MAX;
        if (rel >= 0 && rel < maxlen - off) {   // (LEAD is whole lanes' stretches: no lane straddles a + off)
            int pos = first_diff<LBW>(r, t);
            const int32_t lim = maxlen - off - rel;
            if (lim < 4 * LBW && pos > lim) pos = lim;
            if (pos < 4 * LBW) e = off + rel + pos;
        }
        const unsigned long long sm = __ballot(e != INT32_MAX);
        if (sm) {
            const int32_t m = lane_val(e, first_lane(sm));
            return m < maxlen ? m : maxlen;
        }
        off += LBV - lead;
    }
    return maxlen;
}

#else
// 16 bytes at byte offset off + 16 lane of an LDS byte array (off lane-uniform): three 8-byte reads
// from the 8-byte aligned base below and one alignment for the whole wave (lane stride 16 bytes:
// ds_read_b64 spreads a lane group over all 64 banks but for one pair -- a 32-byte lane stride,
// as before, put 16 lanes on two banks).  The walk is VALU-bound (~500 VALU per match step on
// chr1): 16 bytes per lane and pass cost about half the instructions of 4-byte reads.
__device__ __forceinline__ void lds16(const uint8_t* lds, int32_t off, uint32_t (&o)[4]) {
    const int32_t a = off + 16 * lane_id();
    const uint2* p = reinterpret_cast<const uint2*>(lds + (a & ~7));
    const uint2 v0 = p[0], v1 = p[1], v2 = p[2];
    const uint32_t sh = (uint32_t)(off & 3);
    uint32_t w[5];
    if (off & 4) { w[0] = v0.y; w[1] = v1.x; w[2] = v1.y; w[3] = v2.x; w[4] = v2.y; }
    else { w[0] = v0.x; w[1] = v0.y; w[2] = v1.x; w[3] = v1.y; w[4] = v2.x; }
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

// first differing byte of R-copy[ra..] and T-copy[tb..] within [0, n) (n when none); whole wave,
// 1 KiB per pass, lane l holding the 16 bytes at 16 l of the pass
__device__ __forceinline__ int32_t lds_first_diff(const uint8_t* rbuf, int32_t ra, const uint8_t* tbuf, int32_t tb, int32_t n) {
    const int lane = lane_id();
    for (int32_t base = 0; base < n; base += 1024) {
        const int32_t lim = n - base - 16 * lane;   // bytes of this lane's 16 inside the range
        int e = 16;
        if (lim > 0) {
            uint32_t r[4], t[4];
            lds16(rbuf, ra + base, r);
            lds16(tbuf, tb + base, t);
            e = first_diff<4>(r, t);
            if (e >= lim) e = 16;
        }
        const unsigned long long m = __ballot(e < 16);
        if (m) {
            const int l = first_lane(m);
            return base + 16 * l + lane_val(e, l);
        }
    }
    return n;
}

// longest common extension of R[a..] and T[b..], at most maxlen bytes (extend_alignment,
// compression.cpp:27-34); whole wave.  First from the LDS copy when both starts lie in it; then from
// HBM, LBV bytes of each per round trip, loaded coalesced (16 bytes per lane and KiB, from 16-byte
// aligned bases at most 15 bytes before the LEAD bytes kept ahead of the stretch) into the copy and
// compared from there.  (Lanes loading their own 32-byte stretches took 18 dword loads per lane and
// step, each touching 16 cache lines: with ~5 walk waves per SIMD the round trips queued to ~10 us.)
__device__ __forceinline__ int32_t wave_lce(const WalkPtrs& A, WalkLds& L, BufPos& B, int32_t a, int32_t b, int32_t maxlen) {
    const int lane = lane_id();
    if (maxlen <= 0) return 0;
    int32_t off = 0;
    if (a >= B.rb0 && b >= B.tb0 && a < B.rb0 + LBV && b < B.tb0 + LBV) {
        int32_t avail = B.rb0 + LBV - a < B.tb0 + LBV - b ? B.rb0 + LBV - a : B.tb0 + LBV - b;
        if (avail > maxlen) avail = maxlen;
        const int32_t e = lds_first_diff(L.rbuf, a - B.rb0, L.tbuf, b - B.tb0, avail);
        if (e < avail || avail >= maxlen) return e;
        off = avail;
    }
    while (off < maxlen) {
        const int32_t lead = (a + off >= LEAD && b + off >= LEAD) ? LEAD : 0;
        const int32_t sa = (a + off - lead) & ~15, sb = (b + off - lead) & ~15;
        static_assert(LBV == 2048, "two KiB of each per step");
        const uint4* gr = reinterpret_cast<const uint4*>(A.R + sa) + lane;
        const uint4* gt = reinterpret_cast<const uint4*>(A.T + sb) + lane;
        const uint4 r0 = gr[0], r1 = gr[64], t0 = gt[0], t1 = gt[64];
        wave_sync();   // the copy's previous readers are done
        {
            uint4* dr = reinterpret_cast<uint4*>(L.rbuf) + lane;
            uint4* dt = reinterpret_cast<uint4*>(L.tbuf) + lane;
            dr[0] = r0; dr[64] = r1;
            dt[0] = t0; dt[64] = t1;
        }
        wave_sync();
        B.rb0 = sa;
        B.tb0 = sb;
        const int32_t ra = a + off - sa, tb = b + off - sb;
        int32_t avail = LBV - (ra > tb ? ra : tb);
        if (avail > maxlen - off) avail = maxlen - off;
        const int32_t e = lds_first_diff(L.rbuf, ra, L.tbuf, tb, avail);
        if (e < avail) return off + e;
        off += avail;
    }
    return maxlen;
}

#endif   // WALK_LCE_V

// the same from HBM only (no copy kept; 2 KiB per round trip)
__device__ int32_t wave_lce_hbm(const uint8_t* __restrict__ R, int32_t a, const uint8_t* __restrict__ T, int32_t b,
                                int32_t maxlen) {
    const int lane = lane_id();
    for (int32_t off = 0; off < maxlen; off += 2048) {
        const int32_t my = off + 32 * lane;
        int32_t e = INT32_MAX;
        if (maxlen - my > 0) {
            uint32_t r[8], t[8];
            loadw<8>(R + a + my, r);
            loadw<8>(T + b + my, t);
            int pos = first_diff32(r, t);
            if (maxlen - my < 32 && pos > maxlen - my) pos = maxlen - my;
            if (pos < 32) e = my + pos;
        }
        const unsigned long long sm = __ballot(e != INT32_MAX);
        if (sm) {
            const int32_t m = lane_val(e, first_lane(sm));
            return m < maxlen ? m : maxlen;
        }
    }
    return maxlen > 0 ? maxlen : 0;
}

// extend_alignment (compression.cpp:27-34) of window candidate c for the target k-mer at y: its
// length, or 0 when only the key's kp bases match (k > KEY_K: then c is no candidate at all)
__device__ __forceinline__ int32_t ext_k(const WalkPtrs& A, WalkLds& L, BufPos& B, int32_t c, int32_t y) {
    const int32_t kp = A.kp;
    int32_t maxlen = A.nR - (c + kp);
    const int32_t mt = A.nT - (y + kp);
    if (mt < maxlen) maxlen = mt;
    const int32_t l = kp + wave_lce(A, L, B, c + kp, y + kp, maxlen);
    return l >= A.k ? l : 0;
}

// ---------------------------------------------------------------------------------------------
// window of P in registers: lane l holds the keys of window indices 4l+q (q < 4), i.e. of the
// reference k-mers starting at lo+4l+q, lo = max(0, P-m), up to hi = min(nR-k, P+m).
// 2m+1 <= 4*64 window positions (m = 100: 201).  Its bytes come from the LDS copy when they lie
// in it.
// ---------------------------------------------------------------------------------------------
// A key no k-mer has: pure keys are < 4^kp <= 2^30 (kp <= 15), exotic ones >= 2^31.  Window slots
// outside the window hold it, so "some slot equals kk" needs no vmask test.
constexpr uint32_t KEY_NONE = 0x40000000u;
struct RegWin {
    int32_t P, lo, n;
    uint32_t key[4];  // KEY_NONE outside the window
    uint32_t vmask;   // bit q: index 4*lane+q is inside the window
};

__device__ __forceinline__ void reg_window(const WalkPtrs& A, int32_t P, RegWin& W, const WalkLds* L = nullptr,
                                           const BufPos* B = nullptr) {
    const int lane = lane_id(), k = A.k;
    W.P = P;
    W.lo = P - A.m < 0 ? 0 : P - A.m;
    const int32_t hi = (P + A.m < A.nR - k) ? P + A.m : A.nR - k;
    W.n = hi - W.lo + 1;
    if (W.n < 0) W.n = 0;
    W.vmask = 0;
    W.key[0] = W.key[1] = W.key[2] = W.key[3] = KEY_NONE;
    const bool lds = L && B->has_r(W.lo, W.n + 20);
    const int i0 = 4 * lane;
    if (i0 >= W.n) return;
    uint32_t w[5];   // 20 bytes >= 3 + k
    loadw_sel<5>(lds, lds ? L->rbuf : nullptr, lds ? W.lo - B->rb0 + i0 : 0, A.R + W.lo + i0, w);
    uint64_t code;
    uint32_t bad;
    pack_codes<5>(w, code, bad);
    const int kp = A.kp;
    const uint32_t MASK = (1u << (2 * kp)) - 1u, KM = (1u << kp) - 1u;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        W.key[q] = (bad >> q) & KM ? exotic_key(A.R + W.lo + i0 + q, kp) : (uint32_t)(code >> (2 * q)) & MASK;
        if (i0 + q < W.n) W.vmask |= 1u << q;
        else W.key[q] = KEY_NONE;
    }
}

// key of the target k-mer at y from its 16 bytes w (loaded by the caller; kp <= 15)
__device__ __forceinline__ uint32_t target_key_w(const WalkPtrs& A, int32_t y, const uint32_t (&w)[4]) {
    const int kp = A.kp;
    uint64_t code;
    uint32_t bad;
    pack_codes<4>(w, code, bad);
    return bad & ((1u << kp) - 1u) ? exotic_key(A.T + y, kp) : (uint32_t)code & ((1u << (2 * kp)) - 1u);
}

// bit q set: window index 4*lane+q holds exactly the key's kp bases T[y..y+kp) (key kk)
__device__ __forceinline__ uint32_t win_match(const WalkPtrs& A, const RegWin& W, uint32_t kk, int32_t y) {
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (((W.vmask >> q) & 1u) && W.key[q] == kk) m |= 1u << q;
    if (m && kk >= KEY_EXOTIC) {   // hash keys: confirm bytes (rare)
        const int32_t c0 = W.lo + 4 * lane_id();
        for (int q = 0; q < 4; q++)
            if (((m >> q) & 1u) && !bytes_eq(A.R + c0 + q, A.T + y, A.kp)) m &= ~(1u << q);
    }
    return m;
}

// some window slot holds key kk (exact for pure keys; exotic ones still need win_match's byte check)
__device__ __forceinline__ bool win_any(const RegWin& W, uint32_t kk) {
    return (W.key[0] == kk) | (W.key[1] == kk) | (W.key[2] == kk) | (W.key[3] == kk);
}

// LDS Bloom filter of the register window's keys (only needed for wide literal scans)
__device__ void bloom_window(const RegWin& W, WalkLds& L) {
    const int lane = lane_id();
    uint4* b4 = reinterpret_cast<uint4*>(L.wbits);
    for (int i = lane; i < (1 << (WFBITS - 5)) / 4; i += 64) b4[i] = make_uint4(0, 0, 0, 0);
    wave_sync();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if ((W.vmask >> q) & 1u) {
            const uint32_t f1 = wf_h1(W.key[q]), f2 = wf_h2(W.key[q]), f3 = wf_h3(W.key[q]);
            atomicOr(&L.wbits[f1 >> 5], 1u << (f1 & 31));
            atomicOr(&L.wbits[f2 >> 5], 1u << (f2 & 31));
            atomicOr(&L.wbits[f3 >> 5], 1u << (f3 & 31));
        }
    }
    wave_sync();
}

// Wide literal scan: first position in [x, end) whose k-mer occurs in the window W, or `end` (1024
// positions per wave step: 16 consecutive per lane, keys by shifting one packed code word; the
// Bloom filter passes a superset, confirmed exactly against the register window in position order).
constexpr int WIDE = 16;   // positions per lane per step (1024 per wave step)
#ifndef WIDE_DEPTH
#define WIDE_DEPTH 1       // steps whose words are in flight ahead of the one tested
#endif
// one step's 1024 positions from base: first hit (exact), or -1
__device__ __forceinline__ int32_t wide_step(const WalkPtrs& A, const WalkLds& L, const RegWin& W, int32_t base, int32_t end,
                                             const uint32_t (&w)[8]) {
    const int lane = lane_id(), k = A.kp;
    const uint32_t MASK = (1u << (2 * k)) - 1u, KM = (1u << k) - 1u;
    const int32_t p0 = base + WIDE * lane;
    uint64_t code;
    uint32_t bad;
    pack_codes<8>(w, code, bad);
    // Bloom test for all 16 positions (independent LDS reads)
    uint32_t cand = 0;
#pragma unroll
    for (int st = 0; st < WIDE; st++) {
        const uint32_t key = (bad >> st) & KM ? KEY_EXOTIC : (uint32_t)(code >> (2 * st)) & MASK;
        const uint32_t f1 = wf_h1(key), f2 = wf_h2(key), f3 = wf_h3(key);
        // exotic k-mers always go to the exact check (their key needs the bytes)
        if (key == KEY_EXOTIC ||
            ((L.wbits[f1 >> 5] >> (f1 & 31)) & (L.wbits[f2 >> 5] >> (f2 & 31)) & (L.wbits[f3 >> 5] >> (f3 & 31)) & 1u))
            cand |= 1u << st;
    }
    const int32_t lim = end - p0;
    if (lim < WIDE) cand &= lim > 0 ? (1u << lim) - 1u : 0u;
    // exact check of the candidates, lanes in position order
    for (unsigned long long hm = __ballot(cand != 0); hm; hm &= hm - 1) {
        const int l = __ffsll((long long)hm) - 1;
        uint32_t c = lane_val(cand, l);
        const uint32_t clo = lane_val((uint32_t)code, l), chi = lane_val((uint32_t)(code >> 32), l);
        const uint32_t cbad = lane_val(bad, l);
        const uint64_t lc = ((uint64_t)chi << 32) | clo;
        while (c) {
            const int st = __ffs((int)c) - 1;
            c &= c - 1;
            const int32_t y = base + WIDE * l + st;
            const uint32_t key = (cbad >> st) & KM ? exotic_key(A.T + y, k) : (uint32_t)(lc >> (2 * st)) & MASK;
            if (__ballot(win_match(A, W, key, y) != 0)) return y;
        }
    }
    return -1;
}

// Wide literal scan: first position in [x, end) whose k-mer occurs in the window W, or `end` (1024
// positions per wave step: 16 consecutive per lane, keys by shifting one packed code word; the
// Bloom filter passes a superset, confirmed exactly against the register window in position order).
// The words of the next WIDE_DEPTH steps are in flight while a step is tested.
__device__ __forceinline__ int32_t wide_scan(const WalkPtrs& A, const WalkLds& L, const RegWin& W, int32_t x, int32_t end) {
    const int lane = lane_id();
    uint32_t w[WIDE_DEPTH][8];   // 32 bytes >= WIDE + k - 1 per step
#pragma unroll
    for (int d = 0; d < WIDE_DEPTH; d++)
        if (x + 64 * WIDE * d < end) loadw<8>(A.T + x + 64 * WIDE * d + WIDE * lane, w[d]);
    for (int32_t base = x; base < end;) {
#pragma unroll
        for (int d = 0; d < WIDE_DEPTH; d++) {
            uint32_t cur[8];
#pragma unroll
            for (int i = 0; i < 8; i++) cur[i] = w[d][i];
            const int32_t nb = base + 64 * WIDE * WIDE_DEPTH;
            if (nb < end) loadw<8>(A.T + nb + WIDE * lane, w[d]);
            const int32_t y = wide_step(A, L, W, base, end, cur);
            if (y >= 0) return y;
            base += 64 * WIDE;
            if (base >= end) return end;
        }
    }
    return end;
}

// Long literal scans (WIDE_RING): the words of the next 3 steps stream into LDS by LDS-DMA while a
// step is tested -- a lone wave scanning a stuck stretch otherwise waits a whole HBM round trip
// per 1024 positions (the register prefetch is one step deep: deeper costs the walk registers it
// spills).  The four 1040-byte ring slots reuse the wave's R'/T' copy (invalidated: after a long
// literal stretch it holds nothing the next step needs).  A slot is read with an inline-asm
// ds_read after a counted vmcnt wait (a plain LDS read behind LDS-DMA gets a vmcnt(0) from the
// compiler, which would drain the prefetch every step).  Every exit drains the DMA first.
#ifndef WIDE_RING
#define WIDE_RING 0
#endif
constexpr int RING_SLOT = 1040;          // 1024 positions + the k - 1 <= 15 bytes after them (16)
constexpr int32_t RING_MIN = 8192;       // scans at least this long take the ring
__device__ __forceinline__ uint8_t* ring_slot(WalkLds& L, int i) {
    return ((i & 2) ? L.tbuf : L.rbuf) + (i & 1) * RING_SLOT;
}
__device__ __forceinline__ void ring_issue(const WalkPtrs& A, WalkLds& L, int i, int32_t base) {
    const int lane = lane_id();
    uint8_t* slot = ring_slot(L, i);
    __builtin_amdgcn_global_load_lds((GVoid*)(A.T + base + 16 * lane), (LVoid*)slot, 16, 0, 0);
    if (lane == 0) __builtin_amdgcn_global_load_lds((GVoid*)(A.T + base + 1024), (LVoid*)(slot + 1024), 16, 0, 0);
}
// wait until at most 2 * ahead LDS-DMA instructions are outstanding (each step issues two)
__device__ __forceinline__ void ring_wait(int ahead) {
    if (ahead >= 3) __builtin_amdgcn_s_waitcnt(0x0F76);
    else if (ahead == 2) __builtin_amdgcn_s_waitcnt(0x0F74);
    else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F72);
    else __builtin_amdgcn_s_waitcnt(0x0F70);
}
__device__ __forceinline__ void ring_read(WalkLds& L, int i, uint32_t (&w)[8]) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t addr = (uint32_t)(size_t)(ring_slot(L, i) + 16 * lane_id());
    v4u a, b;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)" : "=v"(a), "=v"(b) : "v"(addr) : "memory");
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ int32_t wide_scan_ring(const WalkPtrs& A, WalkLds& L, BufPos& B, const RegWin& W, int32_t x, int32_t end) {
    B.rb0 = NO_BUF;   // the copy's space becomes the ring
    B.tb0 = NO_BUF;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (this wave's earlier LDS accesses are done)
    wave_sync();
    const int32_t nsteps = (end - x + 1023) >> 10;
    for (int d = 0; d < 3 && d < nsteps; d++) ring_issue(A, L, d, x + 1024 * d);
    int32_t res = end;
    for (int32_t st = 0; st < nsteps; st++) {
        if (st + 3 < nsteps) ring_issue(A, L, (st + 3) & 3, x + 1024 * (st + 3));
        const int32_t left = nsteps - 1 - st;
        ring_wait(left < 3 ? left : 3);
        uint32_t w[8];
        ring_read(L, st & 3, w);
        const int32_t y = wide_step(A, L, W, x + 1024 * st, end, w);
        if (y >= 0) { res = y; break; }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // no DMA may land in the copy's space later
    wave_sync();
    return res;
}

// ---------------------------------------------------------------------------------------------
// the chunk walk (one wave per chunk)
// ---------------------------------------------------------------------------------------------
__device__ int32_t anchor_diag(const WalkPtrs& A, int32_t y0);   // anchors, below
__device__ __forceinline__ int32_t anchor_diag_f(int32_t nT, const uint8_t* __restrict__ T, const uint64_t* __restrict__ atab, int32_t abits,
                                 uint32_t agen, int32_t y0);
#define ANCHOR_DIAG_KC(y) anchor_diag_f(KC->nT, KC->T, KC->atab, KC->abits, KC->agen, (y))

// The kernel's argument segment, laundered: a field read through it is loaded (s_load) where the
// code reads it, instead of being hoisted to the kernel entry and kept in SGPRs.  k_walk reads its
// cold fields (per-chunk state read before the walk loop or written after it) this way: kept live
// across the loop, ~80 SGPRs of them spilled into VGPR lanes (v_writelane / v_readlane).
typedef const __attribute__((address_space(4))) WalkPtrs* KArgPtr;
__device__ __forceinline__ KArgPtr kargs() {
    KArgPtr p = (KArgPtr)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(p));
    return p;
}
#define KC (kargs())

constexpr int DBG_SLOTS = 16;   // ticks, matches, batches, wides, windows, cands, ext bases, t_win, t_find, t_cand, t_tail
#ifndef WALK_WAVES_PER_EU
#define WALK_WAVES_PER_EU 5
#endif
// nlist_dev (optional): the list length from device memory (a round queued before the host knows it)
// CARRY: the carry launch of a round (list = KC->clist): each listed chunk is walked from its
// predecessor's staged exit and committed here, and the walk carries on while the rule allows.
template <bool DBG, bool CARRY>
__global__ __launch_bounds__(64 * WWPB) __attribute__((amdgpu_waves_per_eu(WALK_WAVES_PER_EU)))
void k_walk(WalkPtrs A, const int32_t* __restrict__ list, int32_t nlist, const int32_t* __restrict__ nlist_dev) {
    __shared__ WalkLds lds_all[WWPB];
    const int w = wave_in_block(), lane = lane_id();
    const int32_t li = (int32_t)blockIdx.x * WWPB + w;
    if (nlist_dev) nlist = *nlist_dev;
    if (CARRY && nlist > A.C) nlist = A.C;
    // the round's frozen list starts empty (also when nothing is listed: a round queued blind)
    if (!CARRY && blockIdx.x == 0 && threadIdx.x == 0 && !KC->scal[9]) KC->scal[5] = 0;
    if (li >= nlist || KC->scal[9]) return;
    WalkLds& L = lds_all[w];
    int32_t j = uni(list[li]);   // (j, lo_j, hi_j ... change when the walk carries on, below)
    const int32_t kind = CARRY ? KIND_FIX : uni(KC->kind[j]);
    int32_t lo_j = chunk_lo(A, j);
    int32_t hi_j = chunk_hi(A, j);
    const int32_t lastk = A.nT - A.k;

    int32_t x, P, n = 0, q = 0, ob, cb = -1, cc = 0;
    bool first_spec = false;
    if (CARRY) {   // entry: the predecessor's staged exit (k_commit has not run yet)
        cb = uni(KC->cur[j]);
        ob = 1 - cb;
        cc = uni(KC->cnt[cb][j]);
        x = uni(KC->newX[j - 1]);
        P = uni(KC->newP[j - 1]);
    } else if (kind == KIND_SPEC) {
        ob = uni(KC->cur[j]);
        x = lo_j;
        // a chunk's first speculation (round 1, or the round after a frozen-first round 1 that
        // walked chunk 0 alone): guess from the anchors, re-seed a stuck guess
        first_spec = uni(KC->usedX[j]) == NEVER;
        if (first_spec) {   // first guess: the anchor vote at the chunk start (anchor_diag)
            int32_t d = ANCHOR_DIAG_KC(lo_j);
            // no vote there (an indel, N run or diverged copy under the 128 probes): vote further
            // into the chunk.  A chunk left without a guess costs a whole serial re-walk next round
            // and delays its successor's settlement by one more round.
            for (int i = 1; d == INVALID && i <= ANCHOR_RETRIES && lo_j + i * ANCHOR_RETRY_STEP < hi_j; i++)
                d = uni(ANCHOR_DIAG_KC(lo_j + i * ANCHOR_RETRY_STEP));
            P = INVALID;
            if (d != INVALID) {
                int64_t gp = (int64_t)lo_j - 1 + d;
                P = (int32_t)(gp < 0 ? 0 : (gp > A.nR - 1 ? A.nR - 1 : gp));
            }
            P = uni(P);
            if (lane == 0) KC->guess[j] = P;
        } else {
            P = uni(KC->guess[j]);   // re-speculation (k_round_respec)
        }
        if (lane == 0) { KC->usedX[j] = lo_j; KC->usedP[j] = P; }
    } else if (kind == KIND_FIX) {   // result is committed (or discarded) by k_commit
        cb = uni(KC->cur[j]);
        ob = 1 - cb;
        cc = uni(KC->cnt[cb][j]);
        x = uni(KC->snapX[j]);
        P = uni(KC->snapP[j]);
    } else {   // resume after an escalation was resolved on the host
        cb = uni(KC->cur[j]);
        ob = 1 - cb;
        cc = uni(KC->cnt[cb][j]);
        x = uni(KC->escX[j]);
        P = uni(KC->escP[j]);
        n = uni(KC->escN[j]);
        q = uni(KC->escQ[j]);
    }
    if (!CARRY) {
        if (lane == 0) KC->status[j] = ST_OK;
    }
    int32_t x_entry = x, P_entry = P;
    const uint64_t dbg_t0 = DBG ? wall_clock64() : 0;
    uint64_t dbg_c[13] = {};   // matches, batches, wides, windows, cands, ext bases, t_win, t_find, t_cand, t_tail,
                               // t_hash, t_wide, wide positions
    uint64_t tq = dbg_t0;
    // per-phase clocks only with SCCG_DEBUG_PHASES (each clock read costs a scalar-memory round trip)
    const bool phases = DBG && A.dbg_phases;
    auto tick = [&](int slot) {
        if (DBG && phases) { const uint64_t t = wall_clock64(); dbg_c[slot] += t - tq; tq = t; }
    };
    if (P == INVALID) {   // speculative chunk without an anchor: nothing to offer
        if (lane == 0) { KC->cnt[ob][j] = 0; KC->exitX[j] = INVALID; KC->exitP[j] = INVALID; }
        return;
    }
    // The trajectory buffers: the main walk keeps their addresses; the carry walk (whose chunk
    // changes) forms them where they are used -- loop-carried, they cost it registers it spills.
    const size_t cap = (size_t)A.cap;
    // (formed where they are used -- every 64 matches -- from the argument segment: kept in
    // registers across the walk loop, these pointers and the other cold fields spilled SGPRs)
#define W_OT (KC->bt[ob] + (size_t)j * cap)
#define W_OP (KC->bp[ob] + (size_t)j * cap)
#define W_OL (KC->bl[ob] + (size_t)j * cap)
#define W_CT (KC->bt[cb] + (size_t)j * cap)
#define W_CP (KC->bp[cb] + (size_t)j * cap)
#define W_CL (KC->bl[cb] + (size_t)j * cap)

    RegWin W;
    W.P = INVALID;
    int32_t bloomP = INVALID;   // P whose window keys are in the LDS Bloom filter (built only for wide scans)
    BufPos B;                   // the LDS copy of R'/T' (see WalkLds)
    int32_t lme = x;   // target index after the last match of this walk (start of the open literal run)
    bool converged = false, escalated = false;
    int32_t scan_end = hi_j < lastk + 1 ? hi_j : lastk + 1;
    // a frozen scan found the first window hit of this P in the chunk: the steps before it are
    // literal (the scan covered every position from the frozen chunk's exit on), so the walk
    // starts there -- the trajectory and exit are those of the walk from x
    if (!CARRY && kind == KIND_FIX && A.skip_hints) {
        const int32_t hy = uni(KC->hintY[j]);
        if (hy > x && hy < scan_end && uni(KC->hintP[j]) == P) x = hy;
    }
    // stale entry (predecessor re-walked in this round): converge within the budget or give up
    const bool stale = !CARRY && A.stale_budget > 0 && kind == KIND_FIX && j > 0 && KC->lround[j - 1] == A.round;
    int32_t budget_end = stale && x + A.stale_budget < scan_end ? x + A.stale_budget : scan_end;
    int32_t old_seedq = cb >= 0 ? uni(KC->seedq[j]) : 0;
    int32_t seed_x = x, seedq = 0;
    bool truncated = false;
    // the previous trajectory (fix-ups), 64 entries at a time in registers: lane i holds entry cq0 + i
    int32_t cq0 = -1, ctv = INT32_MAX, cpv = 0, clv = 0;
    auto load_prev = [&](int32_t from) {
        cq0 = from;
        const int32_t qi = from + lane;
        ctv = qi < cc ? W_CT[qi] : INT32_MAX;
        cpv = qi < cc ? W_CP[qi] : 0;
        clv = qi < cc ? W_CL[qi] : 0;
    };
    if (cb >= 0) load_prev(q);   // issued now, waited for at the first match
    // records of the trajectory not stored yet: entries [rb_n0, n), entry rb_n0 + i in lane i (a store
    // per step would make every later load wait for it: vmcnt counts stores and loads in issue order)
    int32_t rb_n0 = n, rbt = 0, rbp = 0, rbl = 0;
    auto flush_recs = [&]() {
        if (lane < n - rb_n0) { W_OT[rb_n0 + lane] = rbt; W_OP[rb_n0 + lane] = rbp; W_OL[rb_n0 + lane] = rbl; }
        rb_n0 = n;
    };
    // A fix-up whose entry is final (its predecessor is not walked in this round) and that ends at
    // its chunk end without converging hands the next chunk to the round's carry launch, which
    // walks it from that exit and carries on from chunk to chunk in one wave: a run of chunks whose
    // speculation failed is then walked in one round, not one round per chunk.  (The loop below
    // only iterates in the carry instantiation, so the main walk's registers stay as they were.)
    for (;;) {
    while (x < scan_end) {
        if (x >= budget_end) { truncated = true; break; }
        if (DBG) tick(9);
        // the probe: keys of the 64 target positions from x (from the LDS copy when it holds them)
        const int32_t y_l = x + lane;
        const bool valid = y_l < scan_end;
        uint32_t tw[4];
        // (4 KiB readable slack after T: no bound needed for the global load)
        loadw_sel<4>(B.has_t(x, 64 + 16), L.tbuf, y_l - B.tb0, A.T + y_l, tw);
        if (W.P != P) { reg_window(A, P, W, &L, &B); if (DBG) dbg_c[3]++; }
        if (DBG) tick(6);
        if (W.n <= 0) { x = scan_end; break; }
        if (DBG) dbg_c[1]++;
        // ---- literal steps: first y in [x, scan_end) whose k-mer has a candidate in the window
        const uint32_t key_l = valid ? target_key_w(A, y_l, tw) : 0u;
        // (after a mismatch the next k-mer usually hits: typically one or two positions.  A hit
        // needs only "some slot equals the key" -- slots outside the window hold KEY_NONE --; an
        // exotic key's hit is confirmed by win_match's byte compare)
        int hl = -1;
        const int nb = scan_end - x < 64 ? scan_end - x : 64;
        for (int yy = 0; yy < nb; yy++) {
            const uint32_t kk = lane_val(key_l, yy);
            if (__ballot(win_any(W, kk)) && (kk < KEY_EXOTIC || __ballot(win_match(A, W, kk, x + yy) != 0))) {
                hl = yy;
                break;
            }
        }
        if (hl < 0) {
            x = (x + 64 < scan_end) ? x + 64 : scan_end;
            if (x < scan_end) {
                int32_t wend = budget_end;
                if (first_spec) {   // re-seed a stuck first guess (see RESEED_GAP)
                    if (x - (lme > seed_x ? lme : seed_x) >= RESEED_GAP) {
                        seed_x = x;
                        const int32_t d = ANCHOR_DIAG_KC(x);
                        if (d != INVALID) {
                            int64_t np = (int64_t)x - 1 + d;
                            np = np < 0 ? 0 : (np > A.nR - 1 ? A.nR - 1 : np);
                            if ((int32_t)np != P) { P = (int32_t)np; seedq = n; continue; }
                        }
                    }
                    const int32_t cpt = (lme > seed_x ? lme : seed_x) + RESEED_GAP;
                    if (cpt < wend) wend = cpt;
                }
                if (DBG) tick(9);
                if (bloomP != P) { bloom_window(W, L); bloomP = P; }
                if (DBG) tick(10);
                const int32_t x0 = x;
                if (WIDE_RING && wend - x >= RING_MIN) x = wide_scan_ring(A, L, B, W, x, wend);
                else x = wide_scan(A, L, W, x, wend);   // exact: x is a hit (or wend)
                if (DBG) { dbg_c[2]++; dbg_c[12] += x - x0; tick(11); }
            }
            continue;
        }
        const int32_t y = x + hl;
        const uint32_t key = lane_val(key_l, hl);
        if (DBG) tick(7);
        // ---- candidates in the window (compression.cpp:114-130, in-range ones only), extended one
        //      at a time by the whole wave; order-free reduction
        const uint32_t mine = win_match(A, W, key, y);   // bit q: window index 4*lane+q matches
        int32_t bl = 0, bcnt = 0;
        bool bhas0 = false;
        uint64_t bkey = ~0ull;
        int ncand = 0;
        for (int qq = 0; qq < 4; qq++) {
            unsigned long long cm = __ballot((mine >> qq) & 1u);
            while (cm) {
                const int cl_ = __ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const int32_t c = W.lo + 4 * cl_ + qq;
                const int32_t l = ext_k(A, L, B, c, y);   // extend_alignment
                ncand++;
                if (!l) continue;   // (k > KEY_K) only the key's bases match
                if (l > bl) { bl = l; bcnt = 1; bhas0 = (c == 0); bkey = c ? pick_key(c, P) : ~0ull; }
                else if (l == bl) {
                    bcnt++;
                    if (c == 0) bhas0 = true;
                    else { const uint64_t pk = pick_key(c, P); bkey = pk < bkey ? pk : bkey; }
                }
            }
        }
        if (!bcnt) {   // (k > KEY_K) no candidate behind the key hits: a literal step
            x = y + 1;
            continue;
        }
        uint64_t pk;
        if (bcnt >= 2 && bhas0) pk = bkey;
        else { const uint64_t k0 = bhas0 ? pick_key(0, P) : ~0ull; pk = k0 < bkey ? k0 : bkey; }
        const int32_t p = (int32_t)(uint32_t)pk;
        if (p == 0) {   // pn2 == 0: the reference falls back to the ungated (pn1, ln1) (:134-138)
            escalated = true;
            if (lane == 0 && !CARRY) {   // (a carried chunk is left as it was: pending next round)
                if (kind == KIND_SPEC) { KC->cnt[ob][j] = 0; KC->exitX[j] = INVALID; KC->exitP[j] = INVALID; }
                else {
                    KC->status[j] = ST_ESC;
                    KC->escX[j] = y; KC->escP[j] = P; KC->escN[j] = n; KC->escQ[j] = q;
                    atomicAdd(&KC->scal[1], 1);
                }
            }
            break;
        }
        {   // the record goes to lane n - rb_n0's registers; 64 at a time are stored together
            const int slot = n - rb_n0;
            if (lane == slot) { rbt = y; rbp = p; rbl = bl; }
            n++;
            if (slot == 63) flush_recs();
        }
        if (DBG) { dbg_c[0]++; dbg_c[4] += ncand; dbg_c[5] += bl; tick(8); }
        // ---- convergence with the previous trajectory of this chunk: q = its first entry with
        //      t >= y (entries are in t order)
        if (cb >= 0) {
            for (;;) {
                if (q >= cq0 + 64) load_prev(q);
                const int32_t qi = cq0 + lane;
                const bool ge = qi >= q && (qi >= cc || ctv >= y);
                const unsigned long long gm = __ballot(ge);
                if (gm) { q = cq0 + first_lane(gm); break; }
                q = cq0 + 64;
            }
            const int ql = q - cq0;
            if (q < cc && q >= old_seedq && lane_val(ctv, ql) == y && lane_val(cpv, ql) == p && lane_val(clv, ql) == bl) {
                flush_recs();
                const int32_t rest = cc - q - 1;
                for (int i = lane; i < rest; i += 64) {
                    W_OT[n + i] = W_CT[q + 1 + i];
                    W_OP[n + i] = W_CP[q + 1 + i];
                    W_OL[n + i] = W_CL[q + 1 + i];
                }
                n += rest;
                rb_n0 = n;   // the copied suffix is stored already
                converged = true;
                break;
            }
        }
        lme = y + bl;
        P = p + bl - 1;   // compression.cpp:149
        x = y + bl;       // compression.cpp:159
    }
    flush_recs();
    if (escalated) return;
    const int32_t nx = converged ? uni(KC->exitX[j]) : x, np = converged ? uni(KC->exitP[j]) : P;
    const bool frozen_end = !converged && x == hi_j && x - lme >= FROZEN_MIN;
    const bool trapped = !converged && x - x_entry >= A.S / 2 && (P - P_entry < TRAP_P && P_entry - P < TRAP_P);
    const bool exit_changed = nx != uni(KC->exitX[j]) || np != uni(KC->exitP[j]);
    if (!CARRY) {
        if (DBG && lane == 0 && (A.dbg_round < 0 || A.dbg_round == A.round)) {
            tick(9);
            uint64_t* d = KC->dbg + (size_t)j * DBG_SLOTS;
            d[0] = wall_clock64() - dbg_t0;
            for (int i = 0; i < 13; i++) d[1 + i] = dbg_c[i];
            d[14] = (uint64_t)A.round;
            d[15] = dbg_t0;   // start (wall clock), for the launch's start spread
        }
        if (lane == 0 && truncated) {   // nothing to commit; the chunk stays pending
            KC->conv[j] = 0;
            KC->changed[j] = 0;
            KC->walked[j] = A.round;
            KC->frozen[j] = 0;
            KC->status[j] = ST_TRUNC;
            return;
        }
        if (lane == 0) {
            KC->cnt[ob][j] = n;
            if (cb < 0) {   // speculative: the trajectory is the chunk's first, take it as is
                KC->exitX[j] = x; KC->exitP[j] = P;
                KC->seedq[j] = seedq;
            } else {        // fix-up: staged; k_commit decides
                KC->newX[j] = nx; KC->newP[j] = np;
                KC->conv[j] = converged;
                KC->changed[j] = exit_changed;
                KC->walked[j] = A.round;
                // ended in a long literal run with P frozen at the chunk end: k_frozen_scan territory
                KC->frozen[j] = frozen_end;
                KC->trapped[j] = trapped;
            }
            KC->status[j] = converged ? ST_CONV : ST_DONE;
        }
        if (truncated) return;
        // carry on only from a fix-up whose commit is certain (k_commit takes it: its predecessor is
        // not listed, and -- by the rule below -- not carried into either), and not where the
        // frozen scan (frozen end) or the trapped re-speculation (k_round_respec) resolves faster
        if (kind != KIND_FIX || (j > 0 && uni(KC->lround[j - 1]) == A.round)) return;
        if (converged || !exit_changed || frozen_end || trapped) return;
        const int32_t j1 = j + 1;
        if (j1 >= A.C || uni(KC->lround[j1]) == A.round || (j1 + 1 < A.C && uni(KC->lround[j1 + 1]) == A.round)) return;
        if (lane == 0) {
            const int32_t at = atomicAdd(&KC->scal[11], 1);
            if (at < A.C) KC->clist[at] = j1;
            atomicOr(&KC->cbits[j1 >> 5], 1u << (j1 & 31));
        }
        return;
    } else {
        // a carried chunk: not on the round's list, so k_commit never sees it -- committed here.
        // A frozen end is left pending (next round's fix-up hands it to the frozen scan).
        if (frozen_end) return;
        if (lane == 0) {
            KC->cnt[ob][j] = n;
            KC->cur[j] = ob;
            KC->exitX[j] = nx; KC->exitP[j] = np;
            KC->usedX[j] = x_entry; KC->usedP[j] = P_entry;
            KC->seedq[j] = 0;
            KC->conv[j] = converged;
            KC->changed[j] = exit_changed;
            KC->walked[j] = A.round;
            KC->frozen[j] = 0;
            KC->trapped[j] = trapped;
        }
    }
    // carry into chunk j + 1 when its entry changed and nobody else walks it or depends on it in
    // this round: j + 1 is not listed, and neither is j + 2 (a listed chunk's predecessor must keep
    // its state for the whole round, so that its own commit rule -- and carry -- stay exact)
    if (converged || !exit_changed || frozen_end || trapped) return;
    const int32_t j1 = j + 1;
    if (j1 >= A.C || uni(KC->lround[j1]) == A.round || (j1 + 1 < A.C && uni(KC->lround[j1 + 1]) == A.round)) return;
    j = j1;
    lo_j = chunk_lo(A, j);
    hi_j = chunk_hi(A, j);
    scan_end = hi_j < lastk + 1 ? hi_j : lastk + 1;
    budget_end = scan_end;
    cb = uni(KC->cur[j]);
    ob = 1 - cb;
    cc = uni(KC->cnt[cb][j]);
    old_seedq = uni(KC->seedq[j]);
    n = 0;
    q = 0;
    rb_n0 = 0;
    seedq = 0;
    converged = false;
    x_entry = x;
    P_entry = P;
    load_prev(0);
    }
}

#undef W_OT
#undef W_OP
#undef W_OL
#undef W_CT
#undef W_CP
#undef W_CL

// Invariant shared by k_commit and the carry launch (k_walk<., true>), which commits the chunks it
// carries into itself: within one round, (1) no chunk is both listed and carried; (2) a carry
// never enters chunk j + 1 when j + 2 is listed (the carried chunk would change a listed chunk's
// predecessor in mid-round); (3) a listed chunk's predecessor is neither listed-and-changed unless
// k_commit sees it (pred_changed below) nor carried (by (2)).  So every commit decision reads a
// predecessor state that is final for the round, and "take a non-converged fix-up only if the
// predecessor did not change" stays exact.  tests/test_gpu_walk_range.py forces long carry chains
// (SCCG_ANCHOR_SHIFT=-2: most speculative guesses wrong) beside frozen and trapped chunks and
// checks every trajectory against the oracle's sequential walk (orc_walk_range).
//
// Commit the fix-ups of a round.  A re-walk that converged is always taken.  One that did not is
// taken only if its predecessor's exit did not change in this round: otherwise its entry was a
// stale (possibly garbage) state and adopting it would push that garbage one chunk further every
// round.  Discarded chunks stay pending and are re-walked from the corrected entry.  Exactness
// never depends on this choice -- the loop only ends when every chunk's trajectory was walked from
// its predecessor's final exit.
__global__ void k_commit(WalkPtrs A, const int32_t* __restrict__ list, int32_t nlist, const int32_t* __restrict__ nlist_dev) {
    if (A.scal[9]) return;   // void pre-queued round
    if (nlist_dev) nlist = *nlist_dev;
    if (blockIdx.x == 0 && threadIdx.x < FROZEN_MAX) A.fy[threadIdx.x] = INT32_MAX;   // for k_frozen_scan
    if (blockIdx.x == 0 && threadIdx.x == 0) A.scal[11] = 0;   // the round's carry list was consumed
    for (int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); i < nlist; i += (int32_t)(gridDim.x * blockDim.x)) {
        const int32_t j = list[i];
        if (A.kind[j] == KIND_SPEC || A.status[j] == ST_ESC || A.status[j] == ST_TRUNC) continue;
        const int32_t round = A.round;
        const bool pred_changed = j > 0 && A.walked[j - 1] == round && A.changed[j - 1];
        if (!(A.conv[j] || !pred_changed)) continue;
        A.cur[j] = 1 - A.cur[j];
        A.exitX[j] = A.newX[j];
        A.exitP[j] = A.newP[j];
        A.usedX[j] = A.snapX[j];
        A.usedP[j] = A.snapP[j];
        A.seedq[j] = 0;   // a fix-up (with a converged suffix) is a walk from its entry
        if (A.frozen[j]) {
            A.flist[atomicAdd(&A.scal[5], 1)] = j;
            atomicOr(&A.fbits[j >> 5], 1u << (j & 31));
        }
    }
}

// The round's frozen list and carry list in chunk order (k_commit and k_walk append in atomic
// order, and mark each entry in a chunk bitmap): which chunks the blind frozen batch (FROZEN_FIRST)
// and the later batches take, which chunks the CARRY_GRID carry waves take, and so the round's
// fills and the next pending list, no longer depend on which wave appended first -- the rounds are
// the same on every run, however long the lists.  One block: the bitmap's words in contiguous
// shares per thread, a block scan of their popcounts, the list rewritten in chunk order, the words
// cleared for the next round.
constexpr int LS_T = 256;   // (a block this small starts beside the other context's walk grid)
__global__ __launch_bounds__(LS_T) void k_list_sort(WalkPtrs A, int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                                    uint32_t* __restrict__ bits) {
    if (A.scal[9]) return;
    __shared__ int32_t wsum[LS_T / 64 + 1];
    if (*count <= 0) return;   // (nothing appended: no bit set)
    const int32_t nw = (A.C + 31) >> 5;
    const int32_t per = (nw + LS_T - 1) / LS_T, w0 = (int32_t)threadIdx.x * per;
    const int32_t w1 = w0 + per < nw ? w0 + per : nw;
    int c = 0;
    for (int32_t w = w0; w < w1; w++) c += __popc(bits[w]);
    const int incl = wave_incl_add<int>(c);
    const int wv = (int)(threadIdx.x >> 6), lane = lane_id();
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int i = 0; i < LS_T / 64; i++) { const int x = wsum[i]; wsum[i] = run; run += x; }
    }
    __syncthreads();
    int at = wsum[wv] + incl - c;
    for (int32_t w = w0; w < w1; w++) {
        uint32_t b = bits[w];
        if (!b) continue;
        bits[w] = 0;
        for (; b; b &= b - 1) list[at++] = (w << 5) + __ffs((int)b) - 1;
    }
}

// Frozen chunks (committed fix-ups that ended in a long literal run with P unchanged up to their
// chunk end; k_commit lists them): for each of the first FROZEN_MAX, the first position after its
// exit whose k-mer key occurs in its window of P, over the whole rest of the target (grid.y picks
// the frozen chunk; every wave builds its own copy of the window -- registers and a 2 KiB Bloom
// filter -- and scans a strided share, 1024 positions per wave step, stopping one step after the
// first hit).  Round 4 tried a block-wide variant (one 2^17-bit one-hash LDS prefilter and a key
// table per block, 64 positions per thread and step): exact, but 10-15x slower per batch on the
// T2T-like genome (a 256-chunk batch 10-15 ms against 0.8 ms; profiles/r04/), so this one stays.
// For k > KEY_K a key hit is a superset of a window hit (the first KEY_K bases), which only makes
// the fills conservative.
constexpr unsigned FZ_GRID = 256;
constexpr int FZ_T = SCCG_BLOCK;
__global__ __launch_bounds__(SCCG_BLOCK) void k_frozen_scan(WalkPtrs A, int fbase) {
    __shared__ WalkLds lds_all[WPB];
    if (A.scal[9]) return;   // void pre-queued round
    const int fi = (int)blockIdx.y, f = fbase + fi;
    if (f >= A.scal[5]) return;
    const int32_t j = A.flist[f];
    const int32_t x0 = A.exitX[j], P = A.exitP[j];
    WalkLds& L = lds_all[wave_in_block()];
    RegWin W;
    reg_window(A, P, W);
    if (W.n <= 0) return;
    bloom_window(W, L);
    const int32_t end = A.nT - A.k + 1 < A.xhi ? A.nT - A.k + 1 : A.xhi;   // (a range walk stops at xhi)
    const int64_t gw = (int64_t)blockIdx.x * WPB + wave_in_block(), G = (int64_t)gridDim.x * WPB;
    for (int64_t base = x0 + gw * 64 * WIDE; base < end; base += G * 64 * WIDE) {
        if (base >= (int64_t)__hip_atomic_load(&A.fy[fi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        const int32_t seg_end = base + 64 * WIDE < end ? (int32_t)(base + 64 * WIDE) : end;
        const int32_t y = wide_scan(A, L, W, (int32_t)base, seg_end);
        if (y < seg_end) {
            if (lane_id() == 0) atomicMin(&A.fy[fi], y);
            return;
        }
    }
}

// The frozen fills of a batch: in chunk order, every frozen chunk of the batch not already covered
// settles the chunks wholly before its first window hit y as literal-only: entry (min(lo, lastk+1),
// P), empty trajectory, exit (min(hi, lastk+1), P) -- instead of one chunk per round.  Each fill is
// consistent on its own (no hit before y), so batches may come in any order; the pending check
// accepts a filled chunk only when it matches its predecessor's exit.
// The chunks a frozen chunk j fills are j+1 .. last: exits are nondecreasing in the chunk index, so
// last is the largest q with min(hi_q, lastk+1) <= y, in closed form.  (Round 3 did the fills
// chunk by chunk in one wave: 1-1.8 ms per round on the T2T-like chromosomes.)
__device__ __forceinline__ int32_t fill_last(const WalkPtrs& A, int32_t j, int32_t y) {
    const int32_t lastk1 = A.nT - A.k + 1;
    const int32_t cap = A.xhi < lastk1 ? A.xhi : lastk1;   // the last chunk's exit
    if (y >= cap) return A.C - 1;
    if (y < A.xlo) return j;
    const int32_t q = (y - A.xlo) / A.S - 1;   // xlo + (q + 1) S <= y (every earlier chunk ends before cap)
    return q < j ? j : (q > A.C - 1 ? A.C - 1 : q);
}
// Chunk state before round 1: no trajectory, no exit, never walked; round 1 takes every chunk,
// chunk 0 exact (a fix-up from the first match's end, with an empty trajectory), the others
// speculative.
// DEV: the start state comes from the first-step statistics in fc (the usual case: the target's
// first k-mer has candidates, compression.cpp:64-161 with pme == -1); when they say otherwise,
// chunk 0 gets no entry (its walk is a no-op) and the host redoes the first step and the init.
template <bool DEV>
__global__ void k_walk_init(WalkPtrs A, int32_t startX, int32_t startP) {
    if (DEV && blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long* r = A.fc + 4;
        if (r[8] != 2 && r[0] == 0 && r[4] > 0) {
            const uint64_t k0 = 1ull << 32;   // pick_key(0, -1)
            const uint64_t pk = (r[5] >= 2 && r[6]) ? r[7] : ((r[6] && k0 < r[7]) ? k0 : r[7]);
            startX = (int32_t)r[4];
            startP = (int32_t)(uint32_t)pk + (int32_t)r[4] - 1;
        } else {
            startX = A.nT - A.k + 1;
            startP = INVALID;
        }
    }
    // scal[9]: the pre-queued round 1 is void (its kernels return at once; the host redoes it)
    if (blockIdx.x == 0 && threadIdx.x == 0) A.scal[9] = DEV && startP == INVALID ? 1 : 0;
    for (int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); j < A.C; j += (int32_t)(gridDim.x * blockDim.x)) {
        A.cur[j] = 0;
        A.cnt[0][j] = 0;
        A.cnt[1][j] = 0;
        A.usedX[j] = NEVER;
        A.usedP[j] = NEVER;
        A.exitX[j] = INVALID;
        A.exitP[j] = INVALID;
        A.kind[j] = j ? KIND_SPEC : KIND_FIX;
        A.plist[j] = j;
        A.lround[j] = 1;
        A.seedq[j] = 0;
        A.trapped[j] = 0;
        A.tflag[j] = 0;
        A.hintY[j] = -1;
        // (round numbers restart at 1 every call: a previous call's "walked in round r, exit
        // changed" must not reach k_commit's predecessor test -- the workspace is reused, and
        // stale values made the rounds vary from call to call)
        A.walked[j] = 0;
        A.changed[j] = 0;
        A.conv[j] = 0;
        A.frozen[j] = 0;
    }
    for (int32_t w = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); w <= A.C / 32; w += (int32_t)(gridDim.x * blockDim.x)) {
        A.fbits[w] = 0;
        A.cbits[w] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.scal[0] = 0; A.scal[1] = 0; A.scal[2] = startX; A.scal[3] = startP;
        A.scal[5] = 0;   // frozen count (k_walk resets it too, but a void round's k_walk returns first)
        A.scal[11] = 0;  // carry list
        A.snapX[0] = startX;
        A.snapP[0] = startP;
    }
}

// Frozen-first start (host first step, chunk 0 literal-only for >= FF_MIN_CHUNKS chunks): round 1
// walked chunk 0 alone and the frozen chain settled the stuck stretch after it; every chunk still
// never walked (and not already listed) now gets its first speculation in round 2 -- the chunks of
// the stuck stretch are never speculated onto the true alignment that the stuck walk never takes.
__global__ void k_spec_rest(WalkPtrs A) {
    const int32_t next = A.round + 1;
    for (int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); q < A.C; q += (int32_t)(gridDim.x * blockDim.x)) {
        if (A.usedX[q] != NEVER || A.lround[q] == next) continue;
        A.kind[q] = KIND_SPEC;
        A.lround[q] = next;
        A.plist[atomicAdd(&A.scal[0], 1)] = q;
    }
}

// The end of a round, three launches (one block over all chunks was a latency-bound loop of
// ~70 us per round, the fixed cost the stuck T2T-like pairs pay ~100 times):
//   k_round_fill     one wave: the frozen fills of a batch; resets the pending list and triggers;
//   k_round_pending  grid, one thread per chunk: the chunks whose entry state (predecessor's exit)
//                    differs from the one their trajectory used -> plist, scal[0] (list order is
//                    free: the walk takes the listed chunks in any order);
//   k_round_respec   one block: re-speculation after the trapped triggers the scan found.
constexpr int RESPEC_T = 1024;
// (1) one block: the batch's frozen chunks sorted by chunk (rank sort), and the fills of the ones no
//     earlier fill covers -> fa_j / fa_l / fa_p, count scal[13]; also resets the pending list
__global__ __launch_bounds__(FROZEN_MAX) void k_round_fill(WalkPtrs A, int fbase, int fcap) {
    if (A.scal[9]) return;   // void pre-queued round
    __shared__ int32_t rj[FROZEN_MAX], ry[FROZEN_MAX], sj[FROZEN_MAX], sy[FROZEN_MAX];
    const int t = (int)threadIdx.x;
    int nf = fcap > 0 ? A.scal[5] - fbase : 0;
    if (nf > fcap) nf = fcap;
    if (nf < 0) nf = 0;
    int32_t j = 0, y = 0;
    if (t < nf) { j = A.flist[fbase + t]; y = A.fy[t]; rj[t] = j; ry[t] = y; }
    __syncthreads();
    if (t < nf) {
        int r = 0;
        for (int f = 0; f < nf; f++) r += rj[f] < j || (rj[f] == j && f < t);
        sj[r] = j;
        sy[r] = y;
    }
    __syncthreads();
    if (t == 0) {
        int na = 0;
        int32_t filled_to = -1;
        for (int r = 0; r < nf; r++) {
            const int32_t jr = sj[r];
            if (jr <= filled_to || jr + 1 >= A.C) continue;
            const int32_t last = fill_last(A, jr, sy[r]);
            if (last > jr) { A.fa_j[na] = jr; A.fa_l[na] = last; A.fa_p[na] = A.exitP[jr]; na++; }
            // the chunk holding the hit: a walk in it with this P has only literal steps before sy[r]
            if (last + 1 < A.C && sy[r] != INT32_MAX) { A.hintY[last + 1] = sy[r]; A.hintP[last + 1] = A.exitP[jr]; }
            filled_to = last;
        }
        A.scal[13] = na;
        A.scal[0] = 0;
        A.scal[12] = 0;
    }
}

// (1b) grid, one thread per chunk: apply the fills (ranges disjoint and in chunk order)
__global__ __launch_bounds__(256) void k_round_fillg(WalkPtrs A) {
    if (A.scal[9]) return;
    __shared__ int32_t fj[FROZEN_MAX], fl[FROZEN_MAX], fp[FROZEN_MAX];
    const int na = A.scal[13];
    if (!na) return;
    for (int i = (int)threadIdx.x; i < na; i += 256) { fj[i] = A.fa_j[i]; fl[i] = A.fa_l[i]; fp[i] = A.fa_p[i]; }
    __syncthreads();
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= A.C) return;
    int lo = 0, hi = na;   // entries with fj < q
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (fj[mid] < q) lo = mid + 1; else hi = mid;
    }
    if (lo == 0 || q > fl[lo - 1]) return;
    const int32_t P = fp[lo - 1];
    const int32_t lastk1 = A.nT - A.k + 1;
    const int32_t lo_q = chunk_lo(A, q), hi_q = chunk_hi(A, q);
    A.cnt[A.cur[q]][q] = 0;
    A.usedX[q] = lo_q < lastk1 ? lo_q : lastk1;
    A.usedP[q] = P;
    A.exitX[q] = hi_q < lastk1 ? hi_q : lastk1;
    A.exitP[q] = P;
    A.changed[q] = 0;
    A.seedq[q] = 0;
    A.trapped[q] = 0;
}

__global__ __launch_bounds__(256) void k_round_pending(WalkPtrs A) {
    if (A.scal[9]) return;
    const int32_t next = A.round + 1;
    const int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j >= A.C) return;
    const int32_t ex = j ? A.exitX[j - 1] : A.scal[2];
    const int32_t ep = j ? A.exitP[j - 1] : A.scal[3];
    const int32_t ux = A.usedX[j], up = A.usedP[j], lr = A.lround[j];
    const bool pend = ex != INVALID && !(ex == ux && ep == up);
    if (!pend) {
        if (lr == next) A.lround[j] = A.round;   // listed by an earlier batch of this round
        // A chunk without a trajectory after its first speculation (no anchor vote anywhere in it:
        // a tandem array, whose 32-mers all repeat, or an escalated speculation) waits until its
        // predecessor settles, and a run of them is then resolved one chunk after another.
        // Speculate it instead from the diagonal of the nearest earlier chunk that has an exit
        // (<= UNGUESSED_LOOKBACK back): inside an array the walk keeps to one diagonal, and the
        // window (+-m) around the guess snaps onto it at the first match.  (Exactness is the
        // loop's: speculation only decides what the next rounds re-walk.)  Opt-in
        // (SCCG_UNGUESSED_SPEC=1): on the T2T-like genome a wrong-diagonal speculation feeds the
        // next fix-up a garbage entry whose frozen scan runs to the target's end (chr2 68 ms ->
        // 0.7 s), and the synthetic tandem-array walk (walk_micro.py dense) kept its 55 rounds --
        // its chunks do get votes, onto the wrong copies of the 171-bp unit.
        if (A.unguessed_spec && j > 0 && ux != NEVER && A.exitX[j] == INVALID) {
            int32_t r = -1;
            for (int32_t q = j - 1; q >= 0 && q >= j - UNGUESSED_LOOKBACK; q--)
                if (A.exitX[q] != INVALID) { r = q; break; }
            if (r >= 0) {
                const int64_t d = (int64_t)A.exitP[r] - A.exitX[r] + 1;
                int64_t gp = (int64_t)chunk_lo(A, j) - 1 + d;
                gp = gp < 0 ? 0 : (gp > A.nR - 1 ? A.nR - 1 : gp);
                A.kind[j] = KIND_SPEC;
                A.guess[j] = (int32_t)gp;
                A.lround[j] = next;
                A.plist[atomicAdd(&A.scal[0], 1)] = j;
            }
        }
        return;
    }
    A.snapX[j] = ex;
    A.snapP[j] = ep;
    A.kind[j] = KIND_FIX;
    A.lround[j] = next;
    A.plist[atomicAdd(&A.scal[0], 1)] = j;
    // (k_round_respec takes the first RESPEC_MAX_TRIGGERS in chunk order; a chunk that was a trigger
    // in an earlier pending pass of this round -- before a chain filled its predecessor -- and is
    // not one now is cleared)
    const bool trig = j > 0 && A.trapped[j - 1] && A.walked[j - 1] == A.round;
    A.tflag[j] = trig ? A.round : -1;
    if (trig) atomicAdd(&A.scal[12], 1);
}

// re-speculate the still-speculative chunks after each trapped trigger (see TRAP_P)
__global__ __launch_bounds__(RESPEC_T) void k_round_respec(WalkPtrs A) {
    if (A.scal[9]) return;
    const int ntrig = A.scal[12];
    if (!ntrig) return;
    const int32_t next = A.round + 1;
    __shared__ int32_t trig[RESPEC_MAX_TRIGGERS];
    __shared__ int32_t wsum[RESPEC_T / 64 + 1];
    // the round's triggers in chunk order (the first RESPEC_MAX_TRIGGERS): thread t takes a contiguous
    // share of the chunks, a block scan of the shares' counts places them -- the same set every run
    {
        const int32_t per = (A.C + RESPEC_T - 1) / RESPEC_T, c0 = (int32_t)threadIdx.x * per;
        int cnt = 0;
        // (a trigger must still be pending: a later frozen batch of the same round may have filled it,
        // and a stale trigger's run would overlap an earlier trigger's -- two waves writing different
        // guesses into the same chunks made the rounds vary from run to run)
        for (int32_t q = c0; q < c0 + per && q < A.C; q++) cnt += A.tflag[q] == A.round && A.lround[q] == next;
        const int incl = wave_incl_add<int>(cnt);
        const int w = (int)(threadIdx.x >> 6), lane = lane_id();
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            int run = 0;
            for (int i = 0; i < RESPEC_T / 64; i++) { const int x = wsum[i]; wsum[i] = run; run += x; }
            wsum[RESPEC_T / 64] = run;
        }
        __syncthreads();
        int at = wsum[w] + incl - cnt;
        for (int32_t q = c0; q < c0 + per && q < A.C && at < RESPEC_MAX_TRIGGERS; q++)
            if (A.tflag[q] == A.round && A.lround[q] == next) trig[at++] = q;
        __syncthreads();
    }
    const int nt = wsum[RESPEC_T / 64] < RESPEC_MAX_TRIGGERS ? wsum[RESPEC_T / 64] : RESPEC_MAX_TRIGGERS;
    const int w = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6), lane = lane_id();
    for (int t = w; t < nt; t += nw) {
        const int32_t j = trig[t], P = A.snapP[j];
        for (int32_t q0 = j + 1; q0 <= j + RESPEC_AHEAD && q0 < A.C; q0 += 64) {
            const int32_t q = q0 + lane;
            // every chunk after a pending one is unconfirmed, so replacing its trajectory by another
            // guess never discards settled work; the run stops at the next pending chunk
            const bool ok = q < A.C && q <= j + RESPEC_AHEAD && A.lround[q] != next;
            const unsigned long long okm = __ballot(ok);
            const unsigned long long run = ~okm ? okm & ((1ull << first_lane(~okm)) - 1) : okm;   // up to the first stop
            if ((run >> lane) & 1ull) {
                A.kind[q] = KIND_SPEC;
                A.guess[q] = P;
                A.lround[q] = next;
                A.plist[atomicAdd(&A.scal[0], 1)] = q;
            }
            if (run != ~0ull) break;
        }
    }
}

// the three round-end launches (fcap = 0: the pending scan alone)
int launch_round_end(const WalkPtrs& A, int fbase, int fcap, hipStream_t s) {
    hipLaunchKernelGGL(k_round_fill, dim3(1), dim3(FROZEN_MAX), 0, s, A, fbase, fcap);
    if (fcap > 0) hipLaunchKernelGGL(k_round_fillg, dim3(grid_for(A.C, 256)), dim3(256), 0, s, A);
    hipLaunchKernelGGL(k_round_pending, dim3(grid_for(A.C, 256)), dim3(256), 0, s, A);
    hipLaunchKernelGGL(k_round_respec, dim3(1), dim3(RESPEC_T), 0, s, A);
    SCCG_HIP(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Frozen chains.  After a deletion longer than m the reference walk's P stays near one reference
// window (compression.cpp:83-101 admits only candidates within m of it): every later target
// position is a literal step except rare chance hits, each of which moves P a little.  Resolving
// that one chunk per round costs a round per hit.  Instead, from the exit state of the earliest
// committed frozen chunk:
//   k_chain_scan  (grid)   every target position from x whose k-mer occurs among the reference
//                          k-mers within CH_BAND of P ("band hits"; exact keys, in position order);
//   k_chain_step  (1 wave) the exact walk over those hits: a hit is a step only if its k-mer is in
//                          the window of the current P (the same candidate / extension / selection
//                          code as k_walk); every other position is a literal step, which is exact
//                          as long as the window stays inside the band.  When it leaves the band,
//                          or a block's hits overflowed, the next generation rescans from x.
//   k_chain_fill           the chunks the chain covered get their trajectories and entry / exit
//                          states, so the round tail finds them settled.
// The chain hands back to the chunk rounds (reason 2) when its matches get dense (the walk is
// aligned again), on a pn2 == 0 step, or when its match list is full.
// ---------------------------------------------------------------------------------------------
__global__ void k_chain_init(WalkPtrs A) {
    if (A.scal[9]) return;
    const int lane = lane_id();
    const int nf = A.scal[5];
    // settled: only a frozen chunk before the first pending one (every chunk up to it was walked
    // from its predecessor's final exit), so the chain walks the sequential walk itself
    int32_t pmin = INT32_MAX;
    if (A.ch_settled) {
        const int np = A.scal[0];
        for (int i = lane; i < np; i += 64) { const int32_t q = A.plist[i]; pmin = q < pmin ? q : pmin; }
        pmin = wave_min(pmin);
    }
    int32_t jm = INT32_MAX;
    for (int f = lane; f < nf; f += 64) { const int32_t j = A.flist[f]; jm = j < jm && j < pmin ? j : jm; }
    jm = wave_min(jm);
    if (lane) return;
    if (jm == INT32_MAX) { A.chs[0] = 0; A.chs[4] = -1; A.chs[5] = 0; return; }   // (chs[4] -1: none started)
    const int32_t x0 = A.exitX[jm], P0 = A.exitP[jm];
    A.chs[0] = 1; A.chs[1] = x0; A.chs[2] = P0; A.chs[3] = 0; A.chs[4] = jm; A.chs[5] = 0;
    A.chs[8] = 0; A.chs[9] = x0; A.chs[10] = P0; A.chs[11] = 0; A.chs[12] = 0; A.chs[13] = INT32_MAX;
}

__device__ __forceinline__ uint32_t ch_slot(uint32_t key) { return slot_hash(key, CH_TBITS); }
constexpr uint32_t CH_EMPTY = 0xFFFFFFFFu;

__global__ __launch_bounds__(1024) void k_chain_scan(WalkPtrs A) {
    __shared__ uint32_t tab[1 << CH_TBITS];
    __shared__ int32_t wsum[17];
    __shared__ int32_t trunc_s;
    __shared__ int32_t s_first;
    if (!A.chs[0]) return;
    const int tid = (int)threadIdx.x, lane = lane_id(), w = wave_in_block(), k = A.k;
    const int32_t x = A.chs[1], P = A.chs[2];
    // mode 1 (band hits were dense): the band is the window itself and each block keeps only its
    // first hit -- a find-first over the rest of the target (blocks past a found hit stop)
    const bool first_only = A.chs[12] != 0;
    const int32_t half = first_only ? A.m : CH_BAND;
    const int32_t blo = P - half < 0 ? 0 : P - half;
    const int32_t bhi = P + half < A.nR - k ? P + half : A.nR - k;
    if (blockIdx.x == 0 && tid == 0) { A.chs[6] = blo; A.chs[7] = bhi; }
    // chs[14]: where this generation's bounded span ends before the target's (INT32_MAX: it does not)
    for (int i = tid; i < (1 << CH_TBITS); i += 1024) tab[i] = CH_EMPTY;
    if (tid == 0) trunc_s = INT32_MAX;
    __syncthreads();
    const int kp = A.kp;   // (keys of the first kp bases: hits are a superset for k > KEY_K)
    const uint32_t MASK = (1u << (2 * kp)) - 1u, KM = (1u << kp) - 1u;
    for (int32_t q = blo + tid; q <= bhi; q += 1024) {   // the band's keys
        uint32_t wv[4], bad;
        uint64_t code;
        loadw<4>(A.R + q, wv);
        pack_codes<4>(wv, code, bad);
        uint32_t key = bad & KM ? exotic_key(A.R + q, kp) : (uint32_t)code & MASK;
        if (key == CH_EMPTY) key = CH_EMPTY - 1;   // (exotic hash collision: a superset is fine)
        uint32_t sl = ch_slot(key);
        for (;;) {
            const uint32_t prev = atomicCAS(&tab[sl], CH_EMPTY, key);
            if (prev == CH_EMPTY || prev == key) break;
            sl = (sl + 1) & ((1u << CH_TBITS) - 1);
        }
    }
    __syncthreads();
    auto in_band = [&](uint32_t key) -> bool {
        if (key == CH_EMPTY) key = CH_EMPTY - 1;
        uint32_t sl = ch_slot(key);
        for (;;) {
            const uint32_t v = tab[sl];
            if (v == key) return true;
            if (v == CH_EMPTY) return false;
            sl = (sl + 1) & ((1u << CH_TBITS) - 1);
        }
    };
    const int32_t lastk1 = A.nT - k + 1;
    int64_t total = (int64_t)lastk1 - x;
    // both modes scan at most CH_GRID * CH_FF_SPAN positions per generation (the next one goes on
    // from the first position not covered): a band-mode generation ends as soon as P leaves the
    // band -- after a few chance hits on a stuck stretch -- so scanning the whole rest of the
    // target (round 3) spent ~0.8 ms per generation on a 243 Mb T2T-like target for hits it never used
    if (total > CH_FF_SPAN * CH_GRID) total = CH_FF_SPAN * CH_GRID;
    const int64_t end = (int64_t)x + (total > 0 ? total : 0);   // < lastk1: the next generation goes on from end
    if (blockIdx.x == 0 && tid == 0) A.chs[14] = end < lastk1 ? (int32_t)end : INT32_MAX;
    int64_t span = total > 0 ? (total + CH_GRID - 1) / CH_GRID : 0;
    span = (span + 15) & ~(int64_t)15;
    const int64_t b0 = (int64_t)x + (int64_t)blockIdx.x * span;
    const int64_t b1 = b0 + span < end ? b0 + span : end;
    int32_t* oy = A.chh_y + (size_t)blockIdx.x * CH_HCAP;
    uint32_t* ok = A.chh_k + (size_t)blockIdx.x * CH_HCAP;
    int32_t cnt = 0;
    int64_t covered = b1;   // first position of the span not covered (b1: all of it)
    for (int64_t base = b0; base < b1; base += 16 * 1024) {
        if (first_only) {
            // block-uniform decision: one load of the shared first hit, seen by every wave (a
            // per-thread load could split the block between breaking and meeting the barriers)
            if (tid == 0) s_first = __hip_atomic_load(&A.chs[13], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            const bool stop = base > (int64_t)s_first;
            __syncthreads();   // s_first is rewritten next step
            if (stop) {
                covered = base;   // a hit lies before this block's rest: the step never gets here
                break;
            }
        }
        const int64_t p0 = base + 16 * tid;
        uint32_t mask = 0;
        uint64_t code = 0;
        uint32_t bad = 0;
        if (p0 < b1) {
            uint32_t wv[8];
            loadw<8>(A.T + p0, wv);   // 4 KiB readable slack after T'
            pack_codes<8>(wv, code, bad);
            const int lim = b1 - p0 < 16 ? (int)(b1 - p0) : 16;
            for (int st = 0; st < lim; st++) {
                const uint32_t key = (bad >> st) & KM ? exotic_key(A.T + p0 + st, kp) : (uint32_t)(code >> (2 * st)) & MASK;
                if (in_band(key)) mask |= 1u << st;
            }
        }
        // block-wide exclusive count of the hits before this thread's (threads in position order)
        const int c = __popc(mask);
        const int incl = wave_incl_add(c);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int i = 0; i < 16; i++) { const int t = wsum[i]; wsum[i] = acc; acc += t; }
            wsum[16] = acc;
        }
        __syncthreads();
        int idx = cnt + wsum[w] + incl - c;
        const int tot = wsum[16];
        for (uint32_t m = mask; m; m &= m - 1) {
            const int st = __ffs((int)m) - 1;
            const int32_t y = (int32_t)(p0 + st);
            if (idx < CH_HCAP) {
                oy[idx] = y;
                ok[idx] = (bad >> st) & KM ? exotic_key(A.T + y, kp) : (uint32_t)(code >> (2 * st)) & MASK;
            } else if (idx == CH_HCAP) {
                trunc_s = y;   // the first hit not kept: positions from here on are not covered
            }
            idx++;
        }
        cnt += tot;
        __syncthreads();   // wsum reuse; trunc_s visible
        if (cnt > CH_HCAP) { covered = trunc_s; break; }
        if (first_only && cnt > 0) {   // this block's first hit is kept (the step needs no more)
            const int32_t y0 = oy[0];
            if (tid == 0) atomicMin(&A.chs[13], y0);
            cnt = 1;
            covered = (int64_t)y0 + 1;
            break;
        }
    }
    if (tid == 0) {
        A.chh_n[blockIdx.x] = cnt < CH_HCAP ? cnt : CH_HCAP;
        // (a window that stops before the target's end: the block holding its end reports it as
        // not covered, so the step ends the generation there)
        const bool cut = covered >= b1 && b0 < b1 && b1 == end && end < lastk1;
        A.chh_tr[blockIdx.x] = covered < b1 ? (int32_t)covered : cut ? (int32_t)end : INT32_MAX;
    }
}

// LDS table of the register window's keys (512 slots, <= 256 keys): 64 band hits are tested at once
constexpr int CH_WBITS = 9;
__device__ void chain_wtab_build(const RegWin& W, uint32_t* tab) {
    const int lane = lane_id();
    for (int i = lane; i < (1 << CH_WBITS); i += 64) tab[i] = CH_EMPTY;
    wave_sync();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if ((W.vmask >> q) & 1u) {
            uint32_t key = W.key[q] == CH_EMPTY ? CH_EMPTY - 1 : W.key[q];
            uint32_t sl = slot_hash(key, CH_WBITS);
            for (;;) {
                const uint32_t prev = atomicCAS(&tab[sl], CH_EMPTY, key);
                if (prev == CH_EMPTY || prev == key) break;
                sl = (sl + 1) & ((1u << CH_WBITS) - 1);
            }
        }
    }
    wave_sync();
}
__device__ __forceinline__ bool chain_wtab_has(const uint32_t* tab, uint32_t key) {
    if (key == CH_EMPTY) key = CH_EMPTY - 1;
    uint32_t sl = slot_hash(key, CH_WBITS);
    for (;;) {
        const uint32_t v = tab[sl];
        if (v == key) return true;
        if (v == CH_EMPTY) return false;
        sl = (sl + 1) & ((1u << CH_WBITS) - 1);
    }
}

__global__ __launch_bounds__(64) void k_chain_step(WalkPtrs A) {
    __shared__ WalkLds L;
    __shared__ uint32_t wtab[1 << CH_WBITS];
    if (!A.chs[0]) return;
    const int lane = lane_id(), k = A.k;
    int32_t x = A.chs[1], P = A.chs[2], nm = A.chs[3];
    const int32_t blo = A.chs[6], bhi = A.chs[7];
    RegWin W;
    W.P = INVALID;
    BufPos B;
    int32_t rt = INT32_MIN;   // lane i: target position of the last chain match with index = i (mod CH_DENSE_N)
    int reason = 0;           // 0: next generation, 1: end of the target reached, 2: hand back
    bool gen_end = false;
    int64_t hits = 0;         // band hits of this generation
    int64_t visited = 0;      // of which the step visited
    // Only the blocks with hits or a cut do anything below: their hit counts and cuts are read at
    // once (coalesced, 64 blocks per load) into LDS with a bitmap of them in block order, and the
    // loop visits those blocks alone -- one dependent pair of loads per block of the scan grid
    // (512) was most of a generation's ~0.2 ms on the T2T-like pairs.
    static_assert(CH_GRID % 64 == 0, "blocks per lane");
    __shared__ int32_t s_nh[CH_GRID], s_tr[CH_GRID];
#pragma unroll
    for (int i = 0; i < CH_GRID / 64; i++) {
        const int b = 64 * i + lane;
        s_nh[b] = A.chh_n[b];
        s_tr[b] = A.chh_tr[b];
    }
    wave_sync();
    if (s_nh[0] == 0 && s_tr[0] == INT32_MAX && lane == 0) A.chs[11] = 0;   // (what block 0, without hits or a cut, does below)
    for (int i = 0; i < CH_GRID / 64 && !gen_end && !reason; i++)
    for (uint64_t bm = __ballot(s_nh[64 * i + lane] > 0 || s_tr[64 * i + lane] != INT32_MAX); bm && !gen_end && !reason;
         bm &= bm - 1) {
        const int b = 64 * i + __ffsll((long long)bm) - 1;
        const int32_t nh = s_nh[b], tr = s_tr[b];
        hits += nh;
        const int32_t* hy = A.chh_y + (size_t)b * CH_HCAP;
        const uint32_t* hk = A.chh_k + (size_t)b * CH_HCAP;
        int32_t yv = lane < nh ? hy[lane] : INT32_MAX;
        uint32_t kv = lane < nh ? hk[lane] : 0u;
        for (int32_t i0 = 0; i0 < nh && !gen_end && !reason; i0 += 64) {
            if (visited >= CH_DENSE_HITS) {
                // band hits this dense cost the step more than one find-first generation per match:
                // stop here (every position before this batch's first hit is settled) and switch
                const int32_t y0 = lane_val(yv, 0);
                if (x < y0) x = y0;
                if (lane == 0) A.chs[12] = 1;
                gen_end = true;
                break;
            }
            visited += nh - i0 < 64 ? nh - i0 : 64;
            // the next 64 hits are loaded while these are visited
            const int32_t in = i0 + 64 + lane;
            const int32_t yn = in < nh ? hy[in] : INT32_MAX;
            const uint32_t kn = in < nh ? hk[in] : 0u;
            const int cntl = nh - i0 < 64 ? nh - i0 : 64;
            for (int li = 0; li < cntl;) {
                if (W.P != P) {
                    reg_window(A, P, W, &L, &B);
                    chain_wtab_build(W, wtab);
                }
                if (W.n <= 0) break;
                // the next of these 64 hits (from lane li) whose key is in the window (a superset
                // for hash keys; win_match below is exact)
                const bool cand = lane >= li && lane < cntl && yv >= x && chain_wtab_has(wtab, kv);
                const unsigned long long cmk = __ballot(cand);
                if (!cmk) break;
                const int hl_ = first_lane(cmk);
                li = hl_ + 1;
                const int32_t y = lane_val(yv, hl_);
                const uint32_t key = lane_val(kv, hl_);
                const uint32_t mine = win_match(A, W, key, y);
                if (!__ballot(mine != 0)) continue;
                // ---- the step (as in k_walk: compression.cpp:110-159)
                int32_t bl = 0, bcnt = 0;
                bool bhas0 = false;
                uint64_t bkey = ~0ull;
                for (int qq = 0; qq < 4; qq++) {
                    unsigned long long cm = __ballot((mine >> qq) & 1u);
                    while (cm) {
                        const int cl_ = __ffsll((long long)cm) - 1;
                        cm &= cm - 1;
                        const int32_t c = W.lo + 4 * cl_ + qq;
                        const int32_t l = ext_k(A, L, B, c, y);
                        if (!l) continue;   // (k > KEY_K) only the key's bases match
                        if (l > bl) { bl = l; bcnt = 1; bhas0 = (c == 0); bkey = c ? pick_key(c, P) : ~0ull; }
                        else if (l == bl) {
                            bcnt++;
                            if (c == 0) bhas0 = true;
                            else { const uint64_t pk = pick_key(c, P); bkey = pk < bkey ? pk : bkey; }
                        }
                    }
                }
                if (!bcnt) continue;   // (k > KEY_K) no candidate: a literal step
                uint64_t pk;
                if (bcnt >= 2 && bhas0) pk = bkey;
                else { const uint64_t k0 = bhas0 ? pick_key(0, P) : ~0ull; pk = k0 < bkey ? k0 : bkey; }
                const int32_t p = (int32_t)(uint32_t)pk;
                // pn2 == 0, list full or a trapped (match-rich) chain: the rounds take over at (x, P)
                if (p == 0 || nm >= A.chm_cap || nm >= CH_HANDBACK_N) { reason = 2; break; }
                if (lane == 0) { A.chm_t[nm] = y; A.chm_p[nm] = p; A.chm_l[nm] = bl; }
                const int slot = nm % CH_DENSE_N;
                const int32_t old = lane_val(rt, slot);
                if (lane == slot) rt = y;
                nm++;
                x = y + bl;
                P = p + bl - 1;
                if (nm > CH_DENSE_N && y - old < CH_DENSE_SPAN) { reason = 2; break; }   // aligned again
                const int32_t wlo = P - A.m < 0 ? 0 : P - A.m;
                const int32_t whi = P + A.m < A.nR - k ? P + A.m : A.nR - k;
                if (wlo < blo || whi > bhi) { gen_end = true; break; }   // window left the band
            }
            yv = yn;
            kv = kn;
        }
        if (!gen_end && !reason && tr != INT32_MAX) {   // hits past tr were not kept
            gen_end = true;
            if (x < tr) x = tr;   // every position before tr is settled (a literal step or a visited hit)
            if (tr == A.chs[14]) {
                // the generation's bounded span ended (no overflow): a long stuck stretch, not dense
                // hits -- counting it as an overflow handed every chain longer than two spans back
                // to the rounds (T2T-like genome 0.52 -> 1.1 s)
                if (lane == 0) A.chs[11] = 0;
            } else {
                // band hits this dense twice running: the chunk rounds are the better engine here
                // (find-first generations stop at their first hit by design)
                if (A.chs[11] >= 1 && !A.chs[12]) reason = 2;
                if (lane == 0) A.chs[11] += 1;
            }
        } else if (lane == 0 && b == 0) {
            A.chs[11] = 0;
        }
    }
    if (!gen_end && !reason) reason = 1;
    if (!reason && A.chs[8] + 1 >= CH_MAX_GENS) reason = 2;   // a wandering chain: back to the rounds
    if (lane == 0) {
        // band hits this dense cost the step more than one find-first generation per match
        if (hits > CH_DENSE_HITS) A.chs[12] = 1;
        A.chs[13] = INT32_MAX;
        A.chs[1] = x;
        A.chs[2] = P;
        A.chs[3] = nm;
        A.chs[5] = reason;
        A.chs[0] = reason == 0;
        A.chs[8] += 1;
    }
}

// first chain match with t >= v (chain matches are in t order)
__device__ __forceinline__ int32_t ch_lower(const int32_t* t, int32_t n, int32_t v) {
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (t[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// one wave per chunk after the chain's start chunk that the chain determined
__global__ __launch_bounds__(SCCG_BLOCK) void k_chain_fill(WalkPtrs A) {
    const int32_t reason = A.chs[5];
    if (A.scal[9] || reason == 0) return;
    const int32_t q = (int32_t)blockIdx.x * WPB + wave_in_block();
    const int32_t j0 = A.chs[4];
    if (q <= j0 || q >= A.C) return;
    const int lane = lane_id(), k = A.k;
    const int32_t lastk1 = A.nT - k + 1;
    const int32_t xe = A.chs[1], nm = A.chs[3], x0 = A.chs[9], P0 = A.chs[10];
    const int32_t lo = chunk_lo(A, q), hi = chunk_hi(A, q);
    const int32_t lo_c = lo < lastk1 ? lo : lastk1, hi_c = hi < lastk1 ? hi : lastk1;
    if (reason == 2 && hi_c > xe) return;   // the chain handed back before this chunk's end
    // walk state at a boundary v: after the last chain match starting before v (or the start)
    auto state_at = [&](int32_t v, int32_t vc, int32_t& sx, int32_t& sp, int32_t& i) {
        i = ch_lower(A.chm_t, nm, v);
        int32_t e = x0, pe = P0;
        if (i > 0) { e = A.chm_t[i - 1] + A.chm_l[i - 1]; pe = A.chm_p[i - 1] + A.chm_l[i - 1] - 1; }
        sx = e > vc ? e : vc;
        sp = pe;
    };
    int32_t ux, up, i1, ex, ep, i2;
    state_at(lo, lo_c, ux, up, i1);
    state_at(hi, hi_c, ex, ep, i2);
    const int32_t n = i2 - i1;
    const int32_t b = A.cur[q];
    int32_t* ot = A.bt[b] + (size_t)q * A.cap;
    int32_t* op = A.bp[b] + (size_t)q * A.cap;
    int32_t* ol = A.bl[b] + (size_t)q * A.cap;
    for (int32_t i = lane; i < n; i += 64) { ot[i] = A.chm_t[i1 + i]; op[i] = A.chm_p[i1 + i]; ol[i] = A.chm_l[i1 + i]; }
    if (lane == 0) {
        A.cnt[b][q] = n;
        A.usedX[q] = ux; A.usedP[q] = up;
        A.exitX[q] = ex; A.exitP[q] = ep;
        A.changed[q] = 0; A.seedq[q] = 0; A.trapped[q] = 0; A.frozen[q] = 0;
    }
}

// ---------------------------------------------------------------------------------------------
// anchors: 32-mers at every 32nd R' position -> position (or MULTI); one probe batch per chunk.
// Direct-mapped table, plain stores: a slot (picked by the top hash bits) holds a 32-bit tag --
// other hash bits XOR the call's generation, so stale slots from earlier calls never match and
// the table is never cleared -- and a position.  Pass 1 stores every sample; pass 2 marks a slot
// MULTI when it holds the same tag with another position (a repeated 32-mer).  A sample that
// loses its slot to a different 32-mer is simply missing.  Anchors only seed speculation: a
// wrong or missing one costs a re-walk, never a wrong result.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t x) {   // bijective
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
// 2-bit code of the 32-mer at s (false if it holds a non-ACGT byte); s 16-byte aligned or not
template <bool ALIGNED>
__device__ __forceinline__ bool code32(const uint8_t* s, uint64_t& code) {
    uint32_t w[8];
    if (ALIGNED) {
        const uint4* p = reinterpret_cast<const uint4*>(s);
        const uint4 a = p[0], b = p[1];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else {
        loadw<8>(s, w);
    }
    uint32_t bad;
    pack_codes<8>(w, code, bad);
    return bad == 0;
}

// A slot holds gen:12 | tag:20 | position:32 (the tag: the key's low 20 bits; the slot index is
// its top bits).  A slot is a hit only for the call's generation, so stale slots never need
// clearing (anchor_generation clears the table when the generation wraps).  Samples that share a
// slot: the last plain store wins by default; SCCG_ANCHOR_DET=1 stores with a 64-bit atomicMax, so
// the winner -- and with it the anchor votes, the speculation and the round counts -- no longer
// depends on which wave stores last.
constexpr uint32_t ANCHOR_GEN_MASK = 0xfffu;
__device__ __forceinline__ uint64_t anchor_slot(const WalkPtrs& A, uint64_t key, uint32_t pos) {
    return ((uint64_t)(A.agen & ANCHOR_GEN_MASK) << 52) | ((uint64_t)(uint32_t)(key & 0xfffffu) << 32) | pos;
}
__device__ __forceinline__ bool anchor_hit(const WalkPtrs& A, uint64_t key, uint64_t v) {
    return (v >> 32) == (anchor_slot(A, key, 0) >> 32) && (uint32_t)v != A_MULTI;
}
__device__ __forceinline__ void anchor_put(const WalkPtrs& A, uint64_t key, uint32_t pos) {
    if (A.adet) atomicMax((unsigned long long*)&A.atab[key >> (64 - A.abits)], (unsigned long long)anchor_slot(A, key, pos));
    else A.atab[key >> (64 - A.abits)] = anchor_slot(A, key, pos);   // (SCCG_ANCHOR_DET=0: last writer wins)
}

// pass 1 (mark = false): store every sample; pass 2 (mark = true): flag repeated 32-mers
template <bool MARK>
__global__ void k_anchor_build(WalkPtrs A) {
    const int64_t ns = A.nR >= ANCHOR_K ? ((int64_t)A.nR - ANCHOR_K) / A.astep + 1 : 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = (int32_t)(i * A.astep);
        uint64_t code;
        if (!code32<true>(A.R + p, code)) continue;
        const uint64_t key = mix64(code);
        if (!MARK) {
            anchor_put(A, key, (uint32_t)p);
        } else {   // (MULTI is the largest position: the mark is an atomicMax too)
            const uint64_t v = A.atab[key >> (64 - A.abits)];
            if ((v >> 32) == (anchor_slot(A, key, 0) >> 32) && (uint32_t)v != (uint32_t)p) anchor_put(A, key, A_MULTI);
        }
    }
}

// Whole wave: probe the 256 target positions from y0; each hit on a sampled reference 32-mer
// votes for its diagonal (reference - target position).  The diagonal with the most votes (>= 2;
// a lone hit is often a repeat copy), ties to the earliest; else the earliest; INVALID if none.
// (the table's fields as arguments: k_walk passes them from its argument segment, kargs)
__device__ __forceinline__ int32_t anchor_diag_f(int32_t nT, const uint8_t* __restrict__ T, const uint64_t* __restrict__ atab, int32_t abits,
                                 uint32_t agen, int32_t y0) {
    const int lane = lane_id();
    constexpr int NB = ANCHOR_PROBE_BATCHES;
    const uint64_t tag = ((uint64_t)(agen & ANCHOR_GEN_MASK) << 52);
    int32_t dg[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const int32_t y = y0 + b * 64 + lane;
        dg[b] = INVALID;
        uint64_t code;
        if (y + ANCHOR_K <= nT && code32<false>(T + y, code)) {
            const uint64_t key = mix64(code);
            const uint64_t v = atab[key >> (64 - abits)];
            // (anchor_hit: this call's generation and the key's tag, not a repeated 32-mer)
            if ((v >> 32) == ((tag | ((uint64_t)(uint32_t)(key & 0xfffffu) << 32)) >> 32) && (uint32_t)v != A_MULTI)
                dg[b] = (int32_t)(uint32_t)v - y;
        }
    }
    int32_t g = INVALID, first = INVALID;
    int gv = 1;
    for (int tries = 0; tries < 8; tries++) {
        int32_t d = INVALID;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const unsigned long long m = __ballot(dg[b] != INVALID);
            if (m && d == INVALID) d = __shfl(dg[b], first_lane(m), 64);
        }
        if (d == INVALID) break;
        if (first == INVALID) first = d;
        int votes = 0;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            votes += __popcll(__ballot(dg[b] == d));
            if (dg[b] == d) dg[b] = INVALID;
        }
        if (votes > gv) { g = d; gv = votes; }
    }
    return g == INVALID ? first : g;
}
__device__ int32_t anchor_diag(const WalkPtrs& A, int32_t y0) { return anchor_diag_f(A.nT, A.T, A.atab, A.abits, A.agen, y0); }


// ---------------------------------------------------------------------------------------------
// exact full-reference candidate scans (the ungated first step and the p2 == 0 escalation)
// ---------------------------------------------------------------------------------------------
constexpr int FC_PER_T = 64;

__device__ __forceinline__ int32_t serial_ext(const uint8_t* R, int32_t nR, const uint8_t* T, int32_t nT, int32_t c,
                                              int32_t y, int k) {
    int32_t l = k;
    while (c + l < nR && y + l < nT && R[c + l] == T[y + l]) ++l;
    return l;
}

// Full-reference k-mer sweep: every thread takes FC_PER_T = 64 consecutive start positions, reads
// their 64 + 16 bytes as five aligned 16-byte loads, tests each position's walk key (and whether
// the k-mer holds a non-ACGT byte) with `pred`, then calls `hit` for every position that passed
// (out of the unrolled part).  HBM-bound: R' is read once per sweep.
template <typename Pred, typename Hit, typename Words>
__device__ __forceinline__ void sweep_kmers_w(const uint8_t* __restrict__ R, int64_t npos, int k, Pred&& pred, Hit&& hit,
                                              Words&& words);
template <typename Pred, typename Hit>
__device__ __forceinline__ void sweep_kmers(const uint8_t* __restrict__ R, int64_t npos, int k, Pred&& pred, Hit&& hit) {
    sweep_kmers_w(R, npos, k, pred, hit, [](int64_t, const uint32_t (&)[20], const uint32_t (&)[20], uint32_t) {});
}
// the same, handing every thread's 64-position block (codes cw, non-ACGT masks dw of its 20 words)
// to `words` as well
template <typename Pred, typename Hit, typename Words>
__device__ __forceinline__ void sweep_kmers_w(const uint8_t* __restrict__ R, int64_t npos, int k, Pred&& pred, Hit&& hit,
                                              Words&& words) {
    const uint32_t MASK = (1u << (2 * k)) - 1u, KM = (1u << k) - 1u;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * FC_PER_T;
    for (int64_t p0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * FC_PER_T; p0 < npos; p0 += stride) {
        uint32_t cw[20], dw[20], acc = 0;
        {
            const uint4* src = reinterpret_cast<const uint4*>(R + p0);
            uint32_t w[20];
#pragma unroll
            for (int i = 0; i < 5; i++) {
                const uint4 v = src[i];
                w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
            }
#pragma unroll
            for (int i = 0; i < 20; i++) { cw[i] = swar_codes(w[i], dw[i]); acc |= dw[i]; }
        }
        words(p0, cw, dw, acc);
        uint64_t hits = 0;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint64_t code = 0;
            uint32_t bad = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) code |= (uint64_t)cw[4 * g + i] << (8 * i);
            if (acc) {   // rare: some byte is not A/C/G/T -- re-read the group's words
                const uint4* gp = reinterpret_cast<const uint4*>(R + p0 + 16 * g);
                const uint4 v0 = gp[0], v1 = gp[1];
                const uint32_t gw[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                for (int i = 0; i < 8; i++) { uint32_t d; swar_codes(gw[i], d); bad |= nz_bytes(d) << (4 * i); }
            }
            uint32_t m16 = 0;   // built high position first: shifts by one, no per-bit constants
            if (!acc) {   // (the usual block: every byte A/C/G/T, every k-mer pure -- no per-position test)
#pragma unroll
                for (int st = 15; st >= 0; st--) m16 = (m16 << 1) | (uint32_t)pred((uint32_t)(code >> (2 * st)) & MASK, true);
            } else {
#pragma unroll
                for (int st = 15; st >= 0; st--)
                    m16 = (m16 << 1) | (uint32_t)pred((uint32_t)(code >> (2 * st)) & MASK, ((bad >> st) & KM) == 0);
            }
            hits |= (uint64_t)m16 << (16 * g);
        }
        if (p0 + FC_PER_T > npos) hits &= npos - p0 >= 64 ? ~0ull : ((1ull << (npos - p0)) - 1);
        while (hits) {
            const int b = __ffsll((long long)hits) - 1;
            hits &= hits - 1;
            hit(p0 + b);
        }
    }
}

// pass 0: max extension over all candidates; pass 1: count / has0 / min pick key at that max
__global__ void k_fullc(WalkPtrs A, int32_t y, int32_t P, int pass) {
    const int k = A.k, kp = A.kp;
    const uint8_t* kb = A.T + y;
    const uint32_t key = walk_key(kb, kp);
    const uint32_t lmax = (uint32_t)A.fc[0];
    const bool exo = key >= KEY_EXOTIC;
    sweep_kmers(A.R, (int64_t)A.nR - k + 1, kp, [&](uint32_t code, bool pure) {
        return exo ? !pure : (pure && code == key);   // exotic (or k > kp): candidates confirmed bytewise below
    }, [&](int64_t c) {
        if ((exo || k > kp) && !bytes_eq(A.R + c, kb, k)) return;
        const int32_t l = serial_ext(A.R, A.nR, A.T, A.nT, (int32_t)c, y, k);
        if (pass == 0) atomicMax(&A.fc[0], (unsigned long long)l);
        else if ((uint32_t)l == lmax) {
            atomicAdd(&A.fc[1], 1ull);
            if (c == 0) atomicOr(&A.fc[2], 1ull);
            else atomicMin(&A.fc[3], (unsigned long long)pick_key((int32_t)c, P));
        }
    });
}

// first target position in [x0, x0+nb) whose k-mer occurs anywhere in R' (pure keys), and the
// first position in the batch holding a non-ACGT k-mer (checked separately, exactly)
constexpr int PB = 1024;
constexpr int PBBITS = 11;
constexpr int PRESENCE_GRID = 1024;   // blocks of a presence sweep (each first builds the batch's LDS tables)
constexpr int KEY0_GRID_MAX = 16384;  // blocks of the first-step sweep (no LDS tables: as many as pay)
constexpr int PFBITS = 17;   // presence pre-filter: 2^17-bit LDS bitmap of the batch's keys

// candidate statistics of one target position (compression.cpp:114-130 over ALL candidates):
// longest extension, how many reach it, whether position 0 does, least pick key among the others
struct CandBest {
    uint32_t l, cnt, has0;
    uint64_t minkey;
};
__device__ __forceinline__ CandBest cb_merge(const CandBest& a, const CandBest& b) {
    if (a.l > b.l) return a;
    if (b.l > a.l) return b;
    return CandBest{a.l, a.cnt + b.cnt, a.has0 | b.has0, a.minkey < b.minkey ? a.minkey : b.minkey};
}
__device__ __forceinline__ CandBest cb_shfl_xor(const CandBest& v, int d) {
    return CandBest{(uint32_t)__shfl_xor((int)v.l, d, 64), (uint32_t)__shfl_xor((int)v.cnt, d, 64),
                    (uint32_t)__shfl_xor((int)v.has0, d, 64), (uint64_t)__shfl_xor((unsigned long long)v.minkey, d, 64)};
}
__device__ __forceinline__ CandBest cb_wave(CandBest v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = cb_merge(v, cb_shfl_xor(v, d));
    return v;
}

// Besides the first batch position with any candidate, the sweep gathers the candidate statistics
// of the batch's FIRST position x0 (the usual answer), so the ungated first step needs no second
// pass: per-block results in fcb, combined by k_cand_reduce into fc[8..11].
__global__ __launch_bounds__(SCCG_BLOCK) void k_presence(WalkPtrs A, int32_t x0, int32_t nb) {
    __shared__ uint32_t hkey[1 << PBBITS];
    __shared__ uint32_t hidx[1 << PBBITS];
    __shared__ uint32_t bits[1 << (PFBITS - 5)];
    __shared__ CandBest wbest[SCCG_BLOCK / 64];
    // keys of the first kp bases: for k > kp the hits are a superset (the host confirms the first
    // with k_fullc) and x0's statistics confirm the rest of each candidate bytewise
    const int k = A.k, kp = A.kp;
    const uint32_t key0 = walk_key(A.T + x0, kp);   // exotic: no statistics (host falls back)
    CandBest best{0, 0, 0, ~0ull};
    for (int i = threadIdx.x; i < (1 << PBBITS); i += blockDim.x) { hkey[i] = 0xffffffffu; hidx[i] = 0xffffffffu; }
    for (int i = threadIdx.x; i < (1 << (PFBITS - 5)); i += blockDim.x) bits[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        uint32_t w[4], bad;
        uint64_t cw;
        loadw<4>(A.T + x0 + i, w);
        pack_codes<4>(w, cw, bad);
        const uint32_t key = bad & ((1u << kp) - 1u) ? exotic_key(A.T + x0 + i, kp) : (uint32_t)cw & ((1u << (2 * kp)) - 1u);
        if (key >= KEY_EXOTIC) { atomicMin(&A.fc[5], (unsigned long long)(x0 + i)); continue; }
        const uint32_t fb = slot_hash(key, PFBITS);
        atomicOr(&bits[fb >> 5], 1u << (fb & 31));
        int slot = (int)slot_hash(key, PBBITS);
        for (;;) {
            const uint32_t prev = atomicCAS(&hkey[slot], 0xffffffffu, key);
            if (prev == 0xffffffffu || prev == key) { atomicMin(&hidx[slot], (uint32_t)i); break; }
            slot = (slot + 1) & ((1 << PBBITS) - 1);
        }
    }
    __syncthreads();
    // the bitmap test is branch-free per position; the exact probe runs only for bitmap hits
    sweep_kmers(A.R, (int64_t)A.nR - k + 1, kp, [&](uint32_t code, bool pure) {
        const uint32_t fb = slot_hash(code, PFBITS);
        return pure && ((bits[fb >> 5] >> (fb & 31)) & 1u);
    }, [&](int64_t c) {
        uint64_t cw = 0;
        uint32_t bad;
        uint32_t w[4];
        loadw<4>(A.R + c, w);
        pack_codes<4>(w, cw, bad);
        const uint32_t code = (uint32_t)cw & ((1u << (2 * kp)) - 1u);
        if (code == key0 && (k == kp || bytes_eq(A.R + c + kp, A.T + x0 + kp, k - kp))) {
            const uint32_t l = (uint32_t)serial_ext(A.R, A.nR, A.T, A.nT, (int32_t)c, x0, k);
            best = cb_merge(best, CandBest{l, 1u, c == 0 ? 1u : 0u, c ? pick_key((int32_t)c, -1) : ~0ull});
        }
        int slot = (int)slot_hash(code, PBBITS);
        for (;;) {
            const uint32_t hk = hkey[slot];
            if (hk == 0xffffffffu) break;
            if (hk == code) { atomicMin(&A.fc[4], (unsigned long long)(x0 + hidx[slot])); break; }
            slot = (slot + 1) & ((1 << PBBITS) - 1);
        }
    });
    best = cb_wave(best);
    if (lane_id() == 0) wbest[wave_in_block()] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < SCCG_BLOCK / 64; i++) best = cb_merge(best, wbest[i]);
        unsigned long long* o = A.fcb + 4 * blockIdx.x;
        o[0] = best.l; o[1] = best.cnt; o[2] = best.has0; o[3] = best.minkey;
    }
}

// The usual first step: does the target's first k-mer (x0) occur in R' at all, and the candidate
// statistics if so.  One key, no tables: a plain compare per reference position, so this sweep
// runs at streaming speed; k_presence (the general batch search) runs only when it finds nothing.
// ANCH: the same pass also stores the anchor samples (every 32nd or 64th position, astep 32 / 64)
// -- their 2-bit codes are the words the sweep already packed, so the anchor index costs no extra
// read of R'.
template <bool ANCH>
__global__ __launch_bounds__(SCCG_BLOCK) void k_key0(WalkPtrs A, int32_t x0) {
    __shared__ CandBest wbest[SCCG_BLOCK / 64];
    const int k = A.k, kp = A.kp;
    const uint32_t key0 = walk_key(A.T + x0, kp);
    CandBest best{0, 0, 0, ~0ull};
    if (key0 < KEY_EXOTIC || ANCH) {   // exotic: no statistics, the caller falls back to k_presence
        const bool want = key0 < KEY_EXOTIC;
        sweep_kmers_w(A.R, (int64_t)A.nR - k + 1, kp, [&](uint32_t code, bool pure) { return want && pure && code == key0; },
                      [&](int64_t c) {
                          if (k > kp && !bytes_eq(A.R + c + kp, A.T + x0 + kp, k - kp)) return;
                          const uint32_t l = (uint32_t)serial_ext(A.R, A.nR, A.T, A.nT, (int32_t)c, x0, k);
                          best = cb_merge(best, CandBest{l, 1u, c == 0 ? 1u : 0u, c ? pick_key((int32_t)c, -1) : ~0ull});
                      },
                      [&](int64_t p0, const uint32_t (&cw)[20], const uint32_t (&dw)[20], uint32_t acc) {
                          if (!ANCH) return;
                          const int nh = A.astep == 32 ? 2 : 1;   // (samples at p0 and p0 + 32, or p0 only)
#pragma unroll
                          for (int h = 0; h < 2; h++) {
                              const int64_t p = p0 + 32 * h;
                              if (h >= nh || p + ANCHOR_K > A.nR) break;
                              uint64_t code = 0;
                              uint32_t bad = 0;
#pragma unroll
                              for (int i = 0; i < 8; i++) {
                                  code |= (uint64_t)cw[8 * h + i] << (8 * i);
                                  bad |= dw[8 * h + i];
                              }
                              if (acc && bad) continue;
                              const uint64_t key = mix64(code);
                              anchor_put(A, key, (uint32_t)p);
                          }
                      });
    }
    best = cb_wave(best);
    if (lane_id() == 0) wbest[wave_in_block()] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < SCCG_BLOCK / 64; i++) best = cb_merge(best, wbest[i]);
        unsigned long long* o = A.fcb + 4 * blockIdx.x;
        o[0] = best.l; o[1] = best.cnt; o[2] = best.has0; o[3] = best.minkey;
    }
}

// ---------------------------------------------------------------------------------------------
// Early sweep: the anchor samples need only R', and the first step's k-mer is the first k bytes of
// T', which can be read straight off the target FASTA.  So the R' sweep runs as soon as R' exists,
// beside the target's strip: it stores the anchors and the positions of that k-mer (k_sweep_early);
// once T' exists, k_cand_stats extends those positions -- what k_key0 + k_cand_reduce would give.
// fc[12]: 1 = early statistics valid, 2 = not usable (too many positions, exotic key, or the FASTA
// reading disagreed with T') -> the caller runs the full k_key0 sweep.  fc[13]: positions found.
// ---------------------------------------------------------------------------------------------
// The first k bytes of T' (strip + toupper + N erase of the target FASTA, the header line
// [hdr[0], hdr[1]) excluded) within the first `limit` FASTA bytes -> kb[0, k), their count -> kb[KB_COUNT..].
// One block, 16 KiB per step: every thread loads its 64 bytes at once (a chromosome starts with
// ~10 kb of N, which a one-wave byte loop crossed in ~10 dependent steps behind the busy strips).
__global__ __launch_bounds__(SCCG_BLOCK) void k_first_kmer(const uint8_t* __restrict__ fa, int64_t n,
                                                           const int64_t* __restrict__ hdr, int k, int64_t limit,
                                                           uint8_t* __restrict__ kb) {
    __shared__ int64_t tmp[5];
    constexpr int PER = 64;
    const int64_t h = hdr[0], he = hdr[1];
    const int64_t end = n < limit ? n : limit;
    int64_t found = 0;
    for (int64_t base = 0; base < end && found < k; base += (int64_t)SCCG_BLOCK * PER) {
        const int64_t p0 = base + (int64_t)threadIdx.x * PER;
        uint32_t w[PER / 4];
        if (p0 + PER + 4 <= end) {
            loadw<PER / 4>(fa + p0, w);
        } else {
#pragma unroll
            for (int q = 0; q < PER / 4; q++) {
                uint32_t v = 0;
                for (int i = 0; i < 4; i++) {
                    const int64_t p = p0 + 4 * q + i;
                    v |= (uint32_t)(p < end ? fa[p] : (uint8_t)' ') << (8 * i);
                }
                w[q] = v;
            }
        }
        uint64_t keep = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint8_t b = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            const int64_t p = p0 + i;
            const bool kp = p < end && !(p >= h && p < he) && !c_isspace(b) && c_toupper(b) != 'N';
            keep |= (uint64_t)kp << i;
        }
        int64_t total = 0;
        int64_t idx = found + block_excl_add((int64_t)__popcll(keep), tmp, &total);
        for (uint64_t m = keep; m && idx < k; m &= m - 1, idx++) {
            const int i = __ffsll((long long)m) - 1;
            kb[idx] = c_toupper((uint8_t)(w[i >> 2] >> (8 * (i & 3))));
        }
        found += total;
    }
    if (threadIdx.x == 0) *reinterpret_cast<int32_t*>(kb + KB_COUNT) = found < k ? (int32_t)found : k;
}

template <bool ANCH>
__global__ __launch_bounds__(SCCG_BLOCK) void k_sweep_early(WalkPtrs A) {
    const int k = A.k, kp = A.kp;
    const int64_t nR = A.dnR ? *A.dnR : A.nR;   // |R'| (A.nR only bounds it)
    const bool have = *reinterpret_cast<const int32_t*>(A.kb + KB_COUNT) == k;
    const uint32_t key0 = have ? walk_key(A.kb, kp) : KEY_EXOTIC;
    const bool want = key0 < KEY_EXOTIC;
    sweep_kmers_w(A.R, nR - k + 1, kp, [&](uint32_t code, bool pure) { return want && pure && code == key0; },
                  [&](int64_t c) {
                      if (k > kp && !bytes_eq(A.R + c + kp, A.kb + kp, k - kp)) return;
                      const unsigned long long i = atomicAdd(&A.fc[13], 1ull);
                      if (i < (unsigned long long)CAND_CAP) A.cand[i] = (int32_t)c;
                  },
                  [&](int64_t p0, const uint32_t (&cw)[20], const uint32_t (&dw)[20], uint32_t acc) {
                      if (!ANCH) return;
                      const int nh = A.astep == 32 ? 2 : 1;   // (samples at p0 and p0 + 32, or p0 only)
#pragma unroll
                      for (int h = 0; h < 2; h++) {
                          const int64_t p = p0 + 32 * h;
                          if (h >= nh || p + ANCHOR_K > nR) break;
                          uint64_t code = 0;
                          uint32_t bad = 0;
#pragma unroll
                          for (int i = 0; i < 8; i++) {
                              code |= (uint64_t)cw[8 * h + i] << (8 * i);
                              bad |= dw[8 * h + i];
                          }
                          if (acc && bad) continue;
                          const uint64_t key = mix64(code);
                          anchor_put(A, key, (uint32_t)p);
                      }
                  });
}

// after T' exists: statistics of x0 = 0 over the early sweep's positions (as k_key0 +
// k_cand_reduce would leave them in fc[4..11]).  Grid-wide: every wave extends one position at a
// time (wave_lce: 2 KiB per round trip), per-block results go to fcb and k_cand_stats_fin merges
// them -- a repeat-rich first k-mer (hundreds of positions) no longer serialises on one block.
constexpr int CAND_STATS_GRID = 256;
// whole wave (one round trip: lane i compares byte i of the FASTA-read k-mer with T')
__device__ __forceinline__ bool cand_stats_usable(const WalkPtrs& A) {
    const int k = A.k, lane = lane_id();
    const bool head = *reinterpret_cast<const int32_t*>(A.kb + KB_COUNT) == k && A.fc[13] <= (unsigned long long)CAND_CAP &&
                      A.nT >= k;
    const bool same = lane >= k || A.kb[lane] == A.T[lane];   // T' has readable slack past nT
    return head && __ballot(!same) == 0 && walk_key(A.kb, A.kp) < KEY_EXOTIC;
}
__global__ __launch_bounds__(SCCG_BLOCK) void k_cand_stats(WalkPtrs A) {
    __shared__ CandBest wbest[SCCG_BLOCK / 64];
    __shared__ int ok;
    const int k = A.k;
    const unsigned long long cnt = A.fc[13];
    if (threadIdx.x < 64) {
        const bool u = cand_stats_usable(A);
        if (threadIdx.x == 0) ok = u;
    }
    __syncthreads();
    CandBest v{0, 0, 0, ~0ull};
    if (ok) {
        const unsigned long long nw = (unsigned long long)gridDim.x * (SCCG_BLOCK / 64);
        for (unsigned long long i = blockIdx.x * (SCCG_BLOCK / 64) + (threadIdx.x >> 6); i < cnt; i += nw) {
            const int32_t c = A.cand[i];
            int32_t maxlen = A.nR - (c + k);
            if (A.nT - k < maxlen) maxlen = A.nT - k;
            const uint32_t l = (uint32_t)(k + wave_lce_hbm(A.R, c + k, A.T, k, maxlen));
            v = cb_merge(v, CandBest{l, 1u, c == 0 ? 1u : 0u, c ? pick_key(c, -1) : ~0ull});
        }
    }
    if (lane_id() != 0) v = CandBest{0, 0, 0, ~0ull};   // the wave's lanes hold the same value: keep one
    v = cb_wave(v);
    if (lane_id() == 0) wbest[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < SCCG_BLOCK / 64; i++) v = cb_merge(v, wbest[i]);
        unsigned long long* o = A.fcb + 4 * blockIdx.x;
        o[0] = v.l; o[1] = v.cnt; o[2] = v.has0; o[3] = v.minkey;
    }
}

__global__ __launch_bounds__(1024) void k_cand_stats_fin(WalkPtrs A, int nblk) {
    __shared__ CandBest wbest[16];
    __shared__ int ok;
    if (threadIdx.x < 64) {
        const bool u = cand_stats_usable(A);
        if (threadIdx.x == 0) { ok = u; A.fc[12] = u ? 1 : 2; }
    }
    __syncthreads();
    if (!ok) return;
    CandBest v{0, 0, 0, ~0ull};
    for (int b = (int)threadIdx.x; b < nblk; b += (int)blockDim.x) {
        const unsigned long long* o = A.fcb + 4 * b;
        v = cb_merge(v, CandBest{(uint32_t)o[0], (uint32_t)o[1], (uint32_t)o[2], o[3]});
    }
    v = cb_wave(v);
    if (lane_id() == 0) wbest[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); i++) v = cb_merge(v, wbest[i]);
        A.fc[8] = v.l; A.fc[9] = v.cnt; A.fc[10] = v.has0; A.fc[11] = v.minkey;
        A.fc[4] = v.cnt ? 0ull : ~0ull;
        A.fc[5] = ~0ull;
    }
}

// fc[8..11] = statistics merged over the sweep's blocks; with x0 >= 0 (after k_key0) also
// fc[4] = x0 when x0's k-mer has a candidate, fc[5] = none
__global__ __launch_bounds__(1024) void k_cand_reduce(WalkPtrs A, int nblk, int32_t x0) {
    __shared__ CandBest wbest[16];
    CandBest v{0, 0, 0, ~0ull};
    for (int b = (int)threadIdx.x; b < nblk; b += (int)blockDim.x) {
        const unsigned long long* o = A.fcb + 4 * b;
        v = cb_merge(v, CandBest{(uint32_t)o[0], (uint32_t)o[1], (uint32_t)o[2], o[3]});
    }
    v = cb_wave(v);
    if (lane_id() == 0) wbest[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); i++) v = cb_merge(v, wbest[i]);
        A.fc[8] = v.l; A.fc[9] = v.cnt; A.fc[10] = v.has0; A.fc[11] = v.minkey;
        if (x0 >= 0) { A.fc[4] = v.cnt ? (unsigned long long)x0 : ~0ull; A.fc[5] = ~0ull; A.fc[12] = 0; }
    }
}

// ---------------------------------------------------------------------------------------------
// flatten + record text
// ---------------------------------------------------------------------------------------------
__global__ void k_chunk_counts(WalkPtrs A) {
    for (int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); j < A.C; j += (int32_t)(gridDim.x * blockDim.x))
        A.flat_off[j] = A.cnt[A.cur[j]][j];
}

__global__ __launch_bounds__(SCCG_BLOCK) void k_flatten(WalkPtrs A, int32_t first) {
    const int32_t j = (int32_t)blockIdx.x * WPB + wave_in_block();
    if (j >= A.C) return;
    const int lane = lane_id();
    const int32_t b = A.cur[j];
    const int32_t n = A.cnt[b][j];
    const int64_t o = A.flat_off[j] + first;
    const int32_t* t = A.bt[b] + (size_t)j * A.cap;
    const int32_t* p = A.bp[b] + (size_t)j * A.cap;
    const int32_t* l = A.bl[b] + (size_t)j * A.cap;
    for (int i = lane; i < n; i += 64) { A.ft[o + i] = t[i]; A.fp[o + i] = p[i]; A.fl[o + i] = l[i]; }
}

// A long literal stretch of the record text, queued for k_long_copy in pieces of at most
// LONG_PIECE bytes (one wave copies one piece).  Every piece but a stretch's last is LONG_PIECE
// long and every stretch is >= LONG_GAP, so nT / LONG_GAP + nT / LONG_PIECE + 2 entries suffice.
constexpr int64_t LONG_PIECE = 64 * 1024;
__device__ __forceinline__ void queue_long(const WalkPtrs& A, int64_t src, int64_t dst, int64_t len) {
    const int64_t np = (len + LONG_PIECE - 1) / LONG_PIECE;
    const int64_t e = (int64_t)atomicAdd((unsigned long long*)&A.scal64[2], (unsigned long long)np);
    for (int64_t i = 0; i < np && e + i < A.lgap_cap; i++) {
        int64_t* q = A.lgap + 3 * (e + i);
        q[0] = src + i * LONG_PIECE;
        q[1] = dst + i * LONG_PIECE;
        q[2] = len - i * LONG_PIECE < LONG_PIECE ? len - i * LONG_PIECE : LONG_PIECE;
    }
}

// One wave copies n bytes s -> d: byte head up to 16-byte alignment of d, then 16-byte stores fed by
// unaligned dword loads (s needs 4 readable bytes of slack), eight per lane in flight, byte tail.
__device__ __forceinline__ void wave_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int64_t n) {
    const int lane = lane_id();
    int64_t head = (int64_t)((16 - ((uintptr_t)d & 15)) & 15);
    if (head > n) head = n;
    if (lane < head) d[lane] = s[lane];
    s += head; d += head; n -= head;
    const int64_t nb = n >> 4;
    uint4* d4 = reinterpret_cast<uint4*>(d);
    for (int64_t c0 = 0; c0 < nb; c0 += 8 * 64) {
        uint32_t w[8][4];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t c = c0 + u * 64 + lane;
            if (c < nb) loadw<4>(s + 16 * c, w[u]);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t c = c0 + u * 64 + lane;
            if (c < nb) d4[c] = make_uint4(w[u][0], w[u][1], w[u][2], w[u][3]);
        }
    }
    const int64_t t = nb << 4;
    if (t + lane < n) d[t + lane] = s[t + lane];
}

// abs_p: absolute p (the text compress_genome writes before delta_encode, compression.cpp:567)
__global__ void k_match_textlen(WalkPtrs A, int64_t nm, int abs_p) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t pend = i ? A.ft[i - 1] + A.fl[i - 1] : 0;
        const int32_t pprev = i && !abs_p ? A.fp[i - 1] : 0;
        const int32_t d = (int32_t)((uint32_t)A.fp[i] - (uint32_t)pprev);
        A.tlen[i] = (int64_t)(A.ft[i] - pend) + 3 + ndigits_i32(d) + ndigits_i32(A.fl[i]);
    }
}

// One thread per match: its literal gap (short ones by the thread, longer ones by the whole wave,
// LONG_GAP and more queued for k_long_copy's grid) and its "(dp,l)" token.
__global__ __launch_bounds__(SCCG_BLOCK) void k_match_textwrite(WalkPtrs A, int64_t nm, uint8_t* __restrict__ out,
                                                                int abs_p) {
    constexpr int32_t SHORT_GAP = 32;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < nm;
    int32_t pend = 0, gap = 0;
    int64_t o = 0;
    if (valid) {
        pend = i ? A.ft[i - 1] + A.fl[i - 1] : 0;
        gap = A.ft[i] - pend;
        o = A.tlen[i];
        if (gap <= SHORT_GAP)
            for (int32_t q = 0; q < gap; q++) out[o + q] = A.T[pend + q];
    }
    if (valid && gap >= LONG_GAP) queue_long(A, pend, o, gap);   // literal-heavy stretches: k_long_copy
    for (unsigned long long lm = __ballot(valid && gap > SHORT_GAP && gap < LONG_GAP); lm; lm &= lm - 1) {
        const int l = __ffsll((long long)lm) - 1;
        const int32_t gp = __shfl(pend, l, 64), gg = __shfl(gap, l, 64);
        const int64_t go = __shfl(o, l, 64);
        for (int32_t q = lane_id(); q < gg; q += 64) out[go + q] = A.T[gp + q];
    }
    if (valid) {
        uint8_t* d = out + o + gap;
        const int32_t pprev = i && !abs_p ? A.fp[i - 1] : 0;
        *d++ = '(';
        d += write_i32(d, (int32_t)((uint32_t)A.fp[i] - (uint32_t)pprev));
        *d++ = ',';
        d += write_i32(d, A.fl[i]);
        *d = ')';
    }
}

// ---------------------------------------------------------------------------------------------
// Record text straight from the chunks' final trajectories (no flattened match list): the chunks'
// target ranges [usedX, exitX) tile the target (the last one runs to |T'|), so chunk j's text is
// its literal gaps and "(dp,l)" tokens, dp taken against the last match of an earlier chunk (or
// the first step's).  Chunk 0 also carries the first step: T'[0, first_y) and its token.
// ---------------------------------------------------------------------------------------------
struct FirstMatch {
    int32_t y, p, l, valid;
};

// (the text kernels return at once after a void pre-queued round: its chunk state is not a walk's)
__global__ void k_chunk_meta(WalkPtrs A) {
    if (A.scal[9]) return;
    for (int32_t j = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); j < A.C; j += (int32_t)(gridDim.x * blockDim.x)) {
        const int32_t n = A.cnt[A.cur[j]][j];
        A.cprev[j] = n > 0 ? j : -1;   // -> exclusive max-scan: the last earlier chunk with a match
        A.flat_off[j] = n;             // -> exclusive sum: match count
    }
}

// k_chunk_meta + both exclusive scans (+ the long-gap counter reset) in one 1024-thread block, for
// up to CP_MAX chunks: cprev[j] = last chunk before j holding a match (-1: none), flat_off[j] =
// matches of the chunks before j, scal64[0] = all of them, scal64[2] = 0 (three launches fewer at
// the end of every round that queues the record text)
constexpr int CP_PER = 16, CP_MAX = 1024 * CP_PER;
__global__ __launch_bounds__(1024) void k_chunk_prefix(WalkPtrs A) {
    __shared__ int64_t wsum[16], wmax[16];
    if (A.scal[9]) return;
    const int tid = (int)threadIdx.x, lane = lane_id(), w = wave_in_block();
    const int32_t per = (A.C + 1023) / 1024, base = tid * per;
    int64_t n[CP_PER];
    int64_t s = 0, mx = -1;
#pragma unroll
    for (int i = 0; i < CP_PER; i++) {
        const int32_t j = base + i;
        n[i] = (i < per && j < A.C) ? A.cnt[A.cur[j]][j] : 0;
        s += n[i];
        if (n[i] > 0) mx = j;
    }
    // inclusive wave scans, then across the 16 waves
    int64_t is = s, im = mx;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t os = __shfl_up(is, d, 64), om = __shfl_up(im, d, 64);
        if (lane >= d) { is += os; im = om > im ? om : im; }
    }
    if (lane == 63) { wsum[w] = is; wmax[w] = im; }
    __syncthreads();
    int64_t cs = 0, cm = -1;
    for (int i = 0; i < w; i++) { cs += wsum[i]; cm = wmax[i] > cm ? wmax[i] : cm; }
    int64_t es = cs + is - s;                                       // exclusive sum before this thread
    int64_t em = __shfl_up(im, 1, 64);                              // exclusive max before this thread
    if (lane == 0) em = -1;
    em = cm > em ? cm : em;
#pragma unroll
    for (int i = 0; i < CP_PER; i++) {
        const int32_t j = base + i;
        if (i < per && j < A.C) {
            A.flat_off[j] = es;
            A.cprev[j] = em;
            es += n[i];
            if (n[i] > 0) em = j;
        }
    }
    if (tid == 1023) { A.scal64[0] = es; A.scal64[2] = 0; }
}

__device__ __forceinline__ int64_t token_len(int32_t d, int32_t l) { return 3 + ndigits_i32(d) + ndigits_i32(l); }
__device__ __forceinline__ int write_token(uint8_t* o, int32_t d, int32_t l) {
    uint8_t* q = o;
    *q++ = '(';
    q += write_i32(q, d);
    *q++ = ',';
    q += write_i32(q, l);
    *q++ = ')';
    return (int)(q - o);
}

// the usual first step (x0 = 0 has candidates), as k_walk_init<true> resolves it from fc[8..11]
__device__ __forceinline__ FirstMatch first_match_dev(const WalkPtrs& A) {
    const unsigned long long* r = A.fc + 4;
    const uint64_t k0 = 1ull << 32;   // pick_key(0, -1)
    const uint64_t pk = (r[5] >= 2 && r[6]) ? r[7] : ((r[6] && k0 < r[7]) ? k0 : r[7]);
    return FirstMatch{0, (int32_t)(uint32_t)pk, (int32_t)r[4], 1};
}

// wave per chunk: WRITE = false -> ctext[j] = its text bytes; WRITE = true -> the text at ctext[j]
// (F.valid == 2: the first match comes from first_match_dev)
template <bool WRITE>
__global__ __launch_bounds__(SCCG_BLOCK) void k_chunk_text(WalkPtrs A, FirstMatch F, int abs_p, uint8_t* __restrict__ out) {
    constexpr int32_t SHORT_GAP = 32;
    const int32_t j = (int32_t)blockIdx.x * WPB + wave_in_block();
    if (j >= A.C || A.scal[9]) return;
    const int lane = lane_id();
    const int32_t b = A.cur[j], n = A.cnt[b][j];
    const int32_t* tt = A.bt[b] + (size_t)j * A.cap;
    const int32_t* pp = A.bp[b] + (size_t)j * A.cap;
    const int32_t* ll = A.bl[b] + (size_t)j * A.cap;
    const int64_t x0 = A.usedX[j], end = j == A.C - 1 ? (int64_t)A.nT : (int64_t)A.exitX[j];
    if (F.valid == 2) F = first_match_dev(A);   // the device's resolution of the usual first step
    int32_t pprev = F.valid ? F.p : 0;
    if (j > 0) {
        const int64_t q = A.cprev[j];
        if (q >= 0) pprev = A.bp[A.cur[q]][(size_t)q * A.cap + A.cnt[A.cur[q]][q] - 1];
    }
    if (abs_p) pprev = 0;
    int64_t o = WRITE ? A.ctext[j] : 0;   // running output offset (wave-uniform)
    // a literal stretch [src, src + len) at o: the lane / the wave / the whole grid (queued)
    auto literal = [&](int64_t src, int64_t len, int64_t at, bool mine) {
        if (!WRITE) return;
        const bool lng = mine && len >= LONG_GAP, med = mine && len > SHORT_GAP && len < LONG_GAP;
        if (mine && len <= SHORT_GAP)
            for (int64_t q = 0; q < len; q++) out[at + q] = A.T[src + q];
        if (lng) queue_long(A, src, at, len);
        for (unsigned long long lm = __ballot(med); lm; lm &= lm - 1) {
            const int l = __ffsll((long long)lm) - 1;
            const int64_t gs = __shfl(src, l, 64), gl = __shfl(len, l, 64), go = __shfl(at, l, 64);
            for (int64_t q = lane; q < gl; q += 64) out[go + q] = A.T[gs + q];
        }
    };
    if (j == 0 && F.valid) {   // the first step: T'[0, y) + its token (dp against 0)
        literal(0, F.y, o, lane == 0);
        o += F.y;
        if (WRITE && lane == 0) write_token(out + o, F.p, F.l);
        o += token_len(F.p, F.l);
    }
    int64_t last_end = x0;
    for (int32_t b0 = 0; b0 < n; b0 += 64) {
        const int32_t i = b0 + lane;
        const bool valid = i < n;
        int32_t t = 0, p = 0, l = 0, pe = 0, pv = 0;
        if (valid) {
            t = tt[i]; p = pp[i]; l = ll[i];
            pe = i ? tt[i - 1] + ll[i - 1] : (int32_t)x0;
            pv = abs_p ? 0 : (i ? pp[i - 1] : pprev);
        }
        const int32_t d = (int32_t)((uint32_t)p - (uint32_t)pv);
        const int64_t gap = valid ? (int64_t)(t - pe) : 0;
        const int64_t len = valid ? gap + token_len(d, l) : 0;
        const int64_t incl = wave_incl_add(len);
        const int64_t at = o + incl - len;
        literal(pe, gap, at, valid);
        if (WRITE && valid) write_token(out + at + gap, d, l);
        o += __shfl(incl, 63, 64);
        const int32_t lastl = (n - b0 < 64 ? n - b0 : 64) - 1;
        last_end = (int64_t)__shfl(t + l, lastl, 64);
    }
    // the chunk's trailing literal [last_end, end)
    if (end > last_end) {
        literal(last_end, end - last_end, o, lane == 0);
        o += end - last_end;
    }
    if (!WRITE && lane == 0) A.ctext[j] = o;
}

// the queued long literal pieces: one wave per piece
__global__ __launch_bounds__(SCCG_BLOCK) void k_long_copy(WalkPtrs A, uint8_t* __restrict__ out) {
    if (A.scal[9]) return;
    const int64_t ne = A.scal64[2] < A.lgap_cap ? A.scal64[2] : A.lgap_cap;
    const int64_t G = (int64_t)gridDim.x * WPB;
    for (int64_t e = (int64_t)blockIdx.x * WPB + wave_in_block(); e < ne; e += G) {
        const int64_t src = A.lgap[3 * e], dst = A.lgap[3 * e + 1], len = A.lgap[3 * e + 2];
        wave_copy(A.T + src, out + dst, len);
    }
}

// out[0, n) = in[0, n): every wave takes LONG_PIECE-byte pieces
__global__ __launch_bounds__(SCCG_BLOCK) void k_copy(const uint8_t* __restrict__ in, int64_t n, uint8_t* __restrict__ out) {
    const int64_t G = (int64_t)gridDim.x * WPB;
    for (int64_t o = ((int64_t)blockIdx.x * WPB + wave_in_block()) * LONG_PIECE; o < n; o += G * LONG_PIECE)
        wave_copy(in + o, out + o, n - o < LONG_PIECE ? n - o : LONG_PIECE);
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct Carve {
    char* base;
    size_t off, cap;
    template <typename T>
    T* take(size_t n) {
        off = (off + 255) & ~(size_t)255;
        T* p = reinterpret_cast<T*>(base + off);
        off += n * sizeof(T);
        return p;
    }
};

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
int anchor_step() {
    static const int v = [] { const int x = env_int("SCCG_ANCHOR_STEP", ANCHOR_STEP_DEFAULT); return x >= 8 && x <= 1024 ? x : ANCHOR_STEP_DEFAULT; }();
    return v;
}
int anchor_bits(int64_t nR) {
    static const int load = [] { const int x = env_int("SCCG_ANCHOR_LOAD", ANCHOR_LOAD_DEFAULT); return x >= 1 && x <= 16 ? x : ANCHOR_LOAD_DEFAULT; }();
    // SCCG_ANCHOR_SHIFT (tuning runs): the table's size in powers of two away from `load` slots per sample
    static const int shift = [] { const int x = env_int("SCCG_ANCHOR_SHIFT", 0); return x >= -4 && x <= 4 ? x : 0; }();
    int64_t want = load * (nR / anchor_step() + 1);
    int b = 10;
    while ((1ll << b) < want && b < 34) b++;
    b += shift;
    return b < 10 ? 10 : b;
}

WalkPtrs carve(void* ws, size_t ws_bytes, const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int k, int m,
               int S, size_t* used, int abits = 0) {
    WalkPtrs A{};
    Carve c{(char*)ws, 0, ws_bytes};
    A.R = R; A.T = T;
    A.nR = (int32_t)nR; A.nT = (int32_t)nT; A.k = k; A.m = m; A.S = S;
    A.kp = k < KEY_K ? k : KEY_K;
    A.C = (int32_t)((nT + S - 1) / S);
    if (A.C < 1) A.C = 1;
    A.xlo = 0;
    A.xhi = (int32_t)nT;
    A.cap = S / k + 4;
    const size_t C = (size_t)A.C, cap = (size_t)A.cap;
    // front: what depends on R' alone (the early sweep fills it before |T'| is known)
    A.abits = abits ? abits : anchor_bits(nR);   // (an early sweep sized it from a bound of |R'|)
    A.astep = anchor_step();
    {
        static const int multi = env_int("SCCG_ANCHOR_MULTI", 0);
        A.amulti = multi;
    }
    A.atab = c.take<uint64_t>((size_t)1 << A.abits);
    A.fc = c.take<unsigned long long>(16);
    A.fcb = c.take<unsigned long long>(4 * KEY0_GRID_MAX);
    A.cand = c.take<int32_t>(CAND_CAP);
    A.kb = c.take<uint8_t>(64);
    for (int b = 0; b < 2; b++) {
        A.bt[b] = c.take<int32_t>(C * cap);
        A.bp[b] = c.take<int32_t>(C * cap);
        A.bl[b] = c.take<int32_t>(C * cap);
        A.cnt[b] = c.take<int32_t>(C);
    }
    A.cur = c.take<int32_t>(C);
    A.exitX = c.take<int32_t>(C); A.exitP = c.take<int32_t>(C);
    A.usedX = c.take<int32_t>(C); A.usedP = c.take<int32_t>(C);
    A.kind = c.take<int32_t>(C); A.status = c.take<int32_t>(C);
    A.escX = c.take<int32_t>(C); A.escP = c.take<int32_t>(C); A.escN = c.take<int32_t>(C); A.escQ = c.take<int32_t>(C);
    A.snapX = c.take<int32_t>(C); A.snapP = c.take<int32_t>(C);
    A.guess = c.take<int32_t>(C);
    A.plist = c.take<int32_t>(C);
    A.rlist = c.take<int32_t>(C);
    A.clist = c.take<int32_t>(C);
    A.newX = c.take<int32_t>(C); A.newP = c.take<int32_t>(C);
    A.conv = c.take<int32_t>(C); A.changed = c.take<int32_t>(C); A.walked = c.take<int32_t>(C);
    A.lround = c.take<int32_t>(C);
    A.seedq = c.take<int32_t>(C);
    A.trapped = c.take<int32_t>(C);
    A.frozen = c.take<int32_t>(C); A.flist = c.take<int32_t>(C);
    A.fbits = c.take<uint32_t>(C / 32 + 1); A.cbits = c.take<uint32_t>(C / 32 + 1);
    A.fy = c.take<int32_t>(FROZEN_MAX);
    A.scal = c.take<int32_t>(16);
    A.trig = c.take<int32_t>(RESPEC_MAX_TRIGGERS);
    A.tflag = c.take<int32_t>(C);
    A.fa_j = c.take<int32_t>(FROZEN_MAX); A.fa_l = c.take<int32_t>(FROZEN_MAX); A.fa_p = c.take<int32_t>(FROZEN_MAX);
    A.hintY = c.take<int32_t>(C); A.hintP = c.take<int32_t>(C);
    A.skip_hints = env_int("SCCG_SKIP_HINTS", 1);
    A.flat_off = c.take<int64_t>(C + 1);
    const size_t maxm = (size_t)(nT / k + 2);
    A.ft = c.take<int32_t>(maxm); A.fp = c.take<int32_t>(maxm); A.fl = c.take<int32_t>(maxm);
    A.tlen = c.take<int64_t>(maxm + 1);
    A.partial = c.take<int64_t>((size_t)scan_partials_needed((int64_t)(maxm > C ? maxm : C) + 1) + 16);
    A.scal64 = c.take<int64_t>(8);
    A.lgap_cap = nT / LONG_GAP + nT / LONG_PIECE + 2;
    A.lgap = c.take<int64_t>(3 * (size_t)A.lgap_cap);
    A.cprev = c.take<int64_t>(C + 1);
    A.ctext = c.take<int64_t>(C + 1);
    A.chs = c.take<int32_t>(16);
    {
        // k_chain_step hands back at CH_HANDBACK_N matches, so no chain stores more than that
        const int64_t mc = nT / k + 2;
        const int64_t lim = CH_HANDBACK_N + 1 < CHAIN_MCAP ? CH_HANDBACK_N + 1 : CHAIN_MCAP;
        A.chm_cap = (int32_t)(mc < lim ? mc : lim);
    }
    A.chm_t = c.take<int32_t>((size_t)A.chm_cap);
    A.chm_p = c.take<int32_t>((size_t)A.chm_cap);
    A.chm_l = c.take<int32_t>((size_t)A.chm_cap);
    A.chh_y = c.take<int32_t>((size_t)CH_GRID * CH_HCAP);
    A.chh_k = c.take<uint32_t>((size_t)CH_GRID * CH_HCAP);
    A.chh_n = c.take<int32_t>(CH_GRID);
    A.chh_tr = c.take<int32_t>(CH_GRID);
    A.dbg = c.take<uint64_t>(C * DBG_SLOTS);
    *used = c.off;
    return A;
}

// SCCG_DEBUG runs take the instrumented walk
using WalkKernel = void (*)(WalkPtrs, const int32_t*, int32_t, const int32_t*);
WalkKernel walk_kernel(const WalkPtrs& A) { return A.dbg ? k_walk<true, false> : k_walk<false, false>; }
// the round's carry launch (after its k_walk, before k_commit): up to CARRY_GRID * WWPB carry chains
// (chunks past that stay pending for the next round, as without carrying)
constexpr int CARRY_GRID = 256;
int launch_carry(const WalkPtrs& A, hipStream_t s) {
    // the carry candidates in chunk order: which ones the CARRY_GRID waves take when there are more
    // is then the same on every run
    hipLaunchKernelGGL(k_list_sort, dim3(1), dim3(LS_T), 0, s, A, A.clist, (const int32_t*)(A.scal + 11), A.cbits);
    PROF_LAUNCH(PROF_WALK_CARRY, s, (A.dbg ? k_walk<true, true> : k_walk<false, true>), dim3(CARRY_GRID), dim3(64 * WWPB), 0, s, A,
                (const int32_t*)A.clist, 0, (const int32_t*)(A.scal + 11));
    SCCG_HIP(hipGetLastError());
    return 0;
}

struct FullC {
    int64_t lmax;
    int32_t p;
};

int set_u64(unsigned long long* p, std::initializer_list<int64_t> v, hipStream_t s) {
    return dev_set_i64(reinterpret_cast<int64_t*>(p), (int)v.size(), v, s);
}

int run_fullc(WalkPtrs& A, int32_t y, int32_t P, FullC* out, hipStream_t s) {
    int rc = set_u64(A.fc, {0, 0, 0, -1}, s);
    if (rc) return rc;
    const int64_t npos = (int64_t)A.nR - A.k + 1;
    unsigned g = grid_for(npos > 0 ? npos : 1, 256 * FC_PER_T);
    if (g > 8192) g = 8192;
    PROF_LAUNCH(PROF_FULLC, s, k_fullc, dim3(g), dim3(256), 0, s, A, y, P, 0);
    PROF_LAUNCH(PROF_FULLC, s, k_fullc, dim3(g), dim3(256), 0, s, A, y, P, 1);
    SCCG_HIP(hipGetLastError());
    unsigned long long r[4];
    {
        const RbItem it{A.fc, r, (int)sizeof r};
        const int rc = dev_readback(&it, 1, s);
        if (rc) return rc;
    }
    out->lmax = (int64_t)r[0];
    if (r[0] == 0) { out->p = INVALID; return 0; }
    const uint64_t k0 = (uint64_t)(uint32_t)(P < 0 ? -P : P) << 32;   // pick_key(0, P)
    uint64_t pk;
    if (r[1] >= 2 && r[2]) pk = r[3];
    else pk = (r[2] && k0 < r[3]) ? k0 : r[3];
    out->p = (int32_t)(uint32_t)pk;
    return 0;
}

// host vector -> device, completed before returning (the vector may die right after)
int h2d_sync(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return 0;
    SCCG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    SCCG_HIP(hipStreamSynchronize(s));
    return 0;
}

// The frozen chain from the earliest frozen chunk committed in this round (k_chain_*): generations
// are queued CH_GENS_PER_SYNC at a time (a finished chain turns the rest into no-ops), then the
// covered chunks are filled.  *gens: generations run; *trapped: it handed back as a trapped
// (match-rich) chain; *started: false when no frozen chunk qualified (a settled-only march chain
// with no frozen chunk before the first pending one) -- nothing was walked or filled.
int run_chain(WalkPtrs& A, hipStream_t s, int* gens, bool* trapped, bool* started) {
    hipLaunchKernelGGL(k_chain_init, dim3(1), dim3(64), 0, s, A);
    SCCG_HIP(hipGetLastError());
    int32_t st[5] = {0, 0, 0, 0, 0};
    *started = true;
    for (int it = 0;; it++) {
        for (int g = 0; g < CH_GENS_PER_SYNC; g++) {
            hipLaunchKernelGGL(k_chain_scan, dim3(CH_GRID), dim3(1024), 0, s, A);
            hipLaunchKernelGGL(k_chain_step, dim3(1), dim3(64), 0, s, A);
        }
        SCCG_HIP(hipGetLastError());
        const RbItem it0{A.chs, st, (int)sizeof st};
        const int rc = dev_readback(&it0, 1, s);
        if (rc) return rc;
        if (!st[0] && st[4] < 0) {   // no chain started (chs[4] = -1 from k_chain_init)
            *started = false;
            *gens = 0;
            *trapped = false;
            return 0;
        }
        if (!st[0]) break;
        if (it > CH_MAX_GENS / CH_GENS_PER_SYNC + 1) return SCCG_E_INTERNAL;   // k_chain_step caps the generations
    }
    PROF_LAUNCH(PROF_WALK_CHAIN, s, k_chain_fill, dim3(grid_for(A.C, WPB)), dim3(SCCG_BLOCK), 0, s, A);
    SCCG_HIP(hipGetLastError());
    int32_t cs[12];
    {
        const RbItem it1{A.chs, cs, (int)sizeof cs};
        const int rc = dev_readback(&it1, 1, s);
        if (rc) return rc;
    }
    *gens = cs[8];
    *trapped = cs[5] == 2 && cs[3] >= CH_HANDBACK_N;
    if (getenv("SCCG_DEBUG"))
        fprintf(stderr, "[chain] from chunk %d (x %d, P %d): %d generations, %d matches, end x %d P %d, reason %d\n", cs[4], cs[9],
                cs[10], cs[8], cs[3], cs[1], cs[2], cs[5]);
    return 0;
}

// Exact walks that hit the pn2 == 0 sentinel stop with status ST_ESC; the reference then takes the
// ungated (pn1, ln1) over ALL candidates (compression.cpp:124-138): resolve each with the full
// scan, append that match, and resume the walk behind it.  Rare: needs P <= m.
int resolve_escalations(WalkPtrs& A, hipStream_t s, std::vector<int32_t>* resumed) {
    const size_t C = (size_t)A.C;
    std::vector<char> seen(C, 0);
    for (;;) {
        int32_t nesc = 0;
        SCCG_HIP(hipMemcpyAsync(&nesc, A.scal + 1, sizeof nesc, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipStreamSynchronize(s));
        if (!nesc) return 0;
        std::vector<int32_t> st(C), ex(C), ep(C), en(C), cur(C);
        SCCG_HIP(hipMemcpyAsync(st.data(), A.status, C * 4, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipMemcpyAsync(ex.data(), A.escX, C * 4, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipMemcpyAsync(ep.data(), A.escP, C * 4, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipMemcpyAsync(en.data(), A.escN, C * 4, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipMemcpyAsync(cur.data(), A.cur, C * 4, hipMemcpyDeviceToHost, s));
        SCCG_HIP(hipStreamSynchronize(s));
        std::vector<int32_t> rl;
        for (size_t j = 0; j < C; j++) {
            if (st[j] != ST_ESC) continue;
            FullC f;
            int rc = run_fullc(A, ex[j], ep[j], &f, s);
            if (rc) return rc;
            if (f.lmax <= 0) return SCCG_E_INTERNAL;   // a window candidate exists, so C is non-empty
            const int32_t ob = 1 - cur[j];
            const size_t at = j * (size_t)A.cap + (size_t)en[j];
            if ((rc = dev_set_i32(A.bt[ob] + at, 1, {ex[j]}, s)) || (rc = dev_set_i32(A.bp[ob] + at, 1, {f.p}, s)) ||
                (rc = dev_set_i32(A.bl[ob] + at, 1, {(int32_t)f.lmax}, s)) ||
                (rc = dev_set_i32(A.escX + j, 1, {ex[j] + (int32_t)f.lmax}, s)) ||
                (rc = dev_set_i32(A.escP + j, 1, {f.p + (int32_t)f.lmax - 1}, s)) ||
                (rc = dev_set_i32(A.escN + j, 1, {en[j] + 1}, s)) || (rc = dev_set_i32(A.kind + j, 1, {KIND_RESUME}, s)))
                return rc;
            rl.push_back((int32_t)j);
            if (!seen[j]) { seen[j] = 1; resumed->push_back((int32_t)j); }
        }
        int rc = dev_set_i32(A.scal + 1, 1, {0}, s);
        if (rc) return rc;
        if ((rc = h2d_sync(A.rlist, rl.data(), rl.size() * 4, s))) return rc;
        PROF_LAUNCH(PROF_WALK, s, walk_kernel(A), dim3(grid_for((int64_t)rl.size(), WWPB)), dim3(64 * WWPB), 0, s, A,
                    (const int32_t*)A.rlist, (int32_t)rl.size(), (const int32_t*)nullptr);
        SCCG_HIP(hipGetLastError());
    }
}

}  // namespace

size_t walk_workspace_bytes(int64_t nR, int64_t nT, int k, int chunk) {
    size_t used = 0;
    carve(nullptr, 0, nullptr, nR, nullptr, nT, k, 100, chunk, &used);
    if (chunk > FF_CHUNK) {   // room for a frozen-first walk re-chunked to FF_CHUNK
        size_t used2 = 0;
        carve(nullptr, 0, nullptr, nR, nullptr, nT, k, 100, FF_CHUNK, &used2);
        if (used2 > used) used = used2;
    }
    return used + 4096;
}

static thread_local WalkPtrs g_last;
static thread_local int64_t g_last_n = 0;

int global_matches(void* /*ws*/, const int32_t** t, const int32_t** p, const int32_t** l, int64_t* n) {
    *t = g_last.ft; *p = g_last.fp; *l = g_last.fl; *n = g_last_n;
    return 0;
}

#define RC(expr)                      \
    do {                              \
        int rc_ = (expr);             \
        if (rc_) return rc_;          \
    } while (0)

namespace {

// The walk's input-only work -- the first step's key sweep (x0 = 0) and the anchor index with
// every chunk's guess -- depends on R' and T' alone.  global_prepare queues it (no host sync), so
// a caller can run it on a second stream while the local pass decides whether the walk is needed
// at all; global_match_and_emit on the same workspace and inputs then skips it.
struct Prepared {
    const void* ws = nullptr;
    const uint8_t* R = nullptr;
    const uint8_t* T = nullptr;
    int64_t nR = -1, nT = -1;
    int k = 0, m = 0, chunk = 0;
    uint32_t agen = 0;
    int abits = 0;
};
thread_local Prepared g_prep;

struct Early {   // an early sweep queued by global_sweep_early
    const void* ws = nullptr;
    const uint8_t* R = nullptr;
    int64_t nR = -1;   // the bound of |R'| it was sized for
    int k = 0;
    uint32_t agen = 0;
    int abits = 0;
};
thread_local Early g_early;

unsigned first_sweep_grid(const WalkPtrs& A) {
    static const unsigned key0_grid = [] {
        const char* e = getenv("SCCG_KEY0_GRID");
        const int v = e ? atoi(e) : 1024;
        return (unsigned)(v >= 64 && v <= KEY0_GRID_MAX ? v : 1024);
    }();
    return grid_for(A.nR - A.k + 1, 256 * FC_PER_T) > key0_grid ? key0_grid : grid_for(A.nR - A.k + 1, 256 * FC_PER_T);
}

// the anchor table's generation for this call (a fresh workspace is cleared once; afterwards every
// call's generation retires old slots)
// Generations increase per workspace and a slot counts only for the call's own generation
// (anchor_hit), so a table region that held nothing but anchor slots since it was last cleared
// needs no clearing: stale slots carry older generations (skipping the clear relies on that
// generation match, not on the store order).  The table is the workspace's first buffer (carve),
// sized by the call's |R'|; the bytes past a call's table belong to its other buffers, so `clean`
// -- the slots that hold only anchor slots -- shrinks to each call's table, and a larger table, a
// new workspace or the 12-bit generation wrapping clears it once.  (The genome job takes its pairs largest first: one
// clear per lane and step.)
struct AnchorSeen { const uint64_t* tab; size_t clean; uint32_t gen; };
std::mutex g_anchor_mu;
std::map<const void*, AnchorSeen> g_anchor_seen;

int anchor_generation(WalkPtrs& A, const void* ws, hipStream_t s) {
    const size_t n = (size_t)1 << A.abits;
    uint32_t g;
    bool clear;
    {
        std::lock_guard<std::mutex> lk(g_anchor_mu);
        AnchorSeen& e = g_anchor_seen[ws];
        clear = e.tab != A.atab || n > e.clean || e.gen >= ANCHOR_GEN_MASK;
        if (clear) e.gen = 0;
        e.tab = A.atab;
        e.clean = n;
        g = ++e.gen;
    }
    if (clear) SCCG_HIP(hipMemsetAsync(A.atab, 0, n * sizeof(uint64_t), s));
    A.agen = g;
    return 0;
}

int queue_prepare(WalkPtrs& A, const void* ws, hipStream_t s) {
    const int32_t lastk = A.nT - A.k;
    const bool walkable = A.nR >= A.k && lastk >= 0;
    if (!walkable) return 0;
    const unsigned gsweep = first_sweep_grid(A);
    RC(anchor_generation(A, ws, s));
    // the usual first step: x0 = 0's own k-mer (statistics land in fc[4..11]); with the default
    // sample stride the same sweep stores the anchor samples
    const bool fused = A.astep == 32 || A.astep == 64;
    if (fused) PROF_LAUNCH(PROF_ANCHOR, s, k_key0<true>, dim3(gsweep), dim3(SCCG_BLOCK), 0, s, A, 0);
    else hipLaunchKernelGGL(k_key0<false>, dim3(gsweep), dim3(SCCG_BLOCK), 0, s, A, 0);
    hipLaunchKernelGGL(k_cand_reduce, dim3(1), dim3(1024), 0, s, A, (int)gsweep, 0);
    SCCG_HIP(hipGetLastError());
    const int64_t ns = (int64_t)A.nR / A.astep + 1;
    const unsigned ga = grid_for(ns, 256) > 8192 ? 8192 : grid_for(ns, 256);
    if (!fused) PROF_LAUNCH(PROF_ANCHOR, s, k_anchor_build<false>, dim3(ga), dim3(256), 0, s, A);
    if (A.amulti) hipLaunchKernelGGL(k_anchor_build<true>, dim3(ga), dim3(256), 0, s, A);
    // (the chunks' first guesses are voted by the round-1 walk itself: anchor_diag at each chunk start)
    SCCG_HIP(hipGetLastError());
    return 0;
}

WalkPtrs make_ptrs(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk, void* ws,
                   size_t ws_bytes, size_t* used, int abits = 0) {
    WalkPtrs A = carve(ws, ws_bytes, Rp, nRp, Tp, nTp, k, m, chunk, used, abits);
    if (!getenv("SCCG_DEBUG")) A.dbg = nullptr;   // per-chunk counters only in diagnostic runs
    A.dbg_phases = getenv("SCCG_DEBUG_PHASES") != nullptr;
    A.dbg_round = getenv("SCCG_DEBUG_ROUND") ? atoi(getenv("SCCG_DEBUG_ROUND")) : -1;
    static const int32_t sb = [] {
        const char* e = getenv("SCCG_STALE_BUDGET");
        return e ? atoi(e) : STALE_BUDGET_DEFAULT;
    }();
    A.stale_budget = sb;
    // (SCCG_ANCHOR_DET=1: atomicMax slots -- the same votes on every run, but the genome bench's
    // sweep took +1.2 ms per step for the read-modify-writes, and the rounds still vary with the
    // chains' timing-dependent generations; off by default)
    A.adet = env_int("SCCG_ANCHOR_DET", 0);
    static const int32_t ug = getenv("SCCG_UNGUESSED_SPEC") != nullptr;
    A.unguessed_spec = ug;
    return A;
}

}  // namespace

void global_prepare_reset() { g_prep = Prepared{}; g_early = Early{}; }

int global_sweep_early(const uint8_t* Rp, int64_t nRp, const int64_t* d_nRp, const uint8_t* tgt_fa, int64_t tn,
                       const int64_t* d_hdr, int k, int m, int chunk, void* ws, size_t ws_bytes, hipStream_t s) {
    g_early = Early{};
    if (m < 0 || 2 * m + 1 > WCAP || k > KMAX || k < 1) return SCCG_E_UNSUPPORTED;
    if (nRp < k || tn <= 0) return 0;   // no walk can use it
    size_t used = 0;
    // |T'| <= tn: the carve's R'-only front (anchor table, fc, positions, kb) does not depend on it;
    // nRp bounds |R'|, which the sweep reads from d_nRp
    WalkPtrs A = make_ptrs(Rp, nRp, nullptr, tn, k, m, chunk, ws, ws_bytes, &used);
    if (used > ws_bytes) return SCCG_E_INTERNAL;
    A.dnR = d_nRp;
    RC(anchor_generation(A, ws, s));
    RC(set_u64(A.fc + 12, {0, 0}, s));
    hipLaunchKernelGGL(k_first_kmer, dim3(1), dim3(SCCG_BLOCK), 0, s, tgt_fa, tn, d_hdr, k, (int64_t)1 << 20, A.kb);
    const unsigned g = first_sweep_grid(A);
    if (A.astep == 32 || A.astep == 64) {
        PROF_LAUNCH(PROF_ANCHOR, s, k_sweep_early<true>, dim3(g), dim3(SCCG_BLOCK), 0, s, A);
    } else {
        hipLaunchKernelGGL(k_sweep_early<false>, dim3(g), dim3(SCCG_BLOCK), 0, s, A);
        const int64_t ns = (int64_t)A.nR / A.astep + 1;
        const unsigned ga = grid_for(ns, 256) > 8192 ? 8192 : grid_for(ns, 256);
        PROF_LAUNCH(PROF_ANCHOR, s, k_anchor_build<false>, dim3(ga), dim3(256), 0, s, A);
    }
    SCCG_HIP(hipGetLastError());
    g_early = Early{ws, Rp, nRp, k, A.agen, A.abits};
    return 0;
}

int global_prepare(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk, void* ws,
                   size_t ws_bytes, hipStream_t s) {
    g_prep = Prepared{};
    if (m < 0 || 2 * m + 1 > WCAP || k > KMAX || k < 1) return SCCG_E_UNSUPPORTED;
    const Early e = g_early;
    g_early = Early{};
    const bool early = e.ws == ws && e.R == Rp && e.nR >= nRp && e.k == k;
    size_t used = 0;
    WalkPtrs A = make_ptrs(Rp, nRp, Tp, nTp, k, m, chunk, ws, ws_bytes, &used, early ? e.abits : 0);
    if (used > ws_bytes) return SCCG_E_INTERNAL;
    if (early) {
        // the early sweep already stored the anchors and the first k-mer's positions
        A.agen = e.agen;
        if (A.nR >= A.k && A.nT >= A.k) {
            hipLaunchKernelGGL(k_cand_stats, dim3(CAND_STATS_GRID), dim3(SCCG_BLOCK), 0, s, A);
            hipLaunchKernelGGL(k_cand_stats_fin, dim3(1), dim3(1024), 0, s, A, CAND_STATS_GRID);
            if (A.amulti) {
                const int64_t ns = (int64_t)A.nR / A.astep + 1;
                const unsigned ga = grid_for(ns, 256) > 8192 ? 8192 : grid_for(ns, 256);
                hipLaunchKernelGGL(k_anchor_build<true>, dim3(ga), dim3(256), 0, s, A);
            }
            SCCG_HIP(hipGetLastError());
        }
    } else {
        RC(queue_prepare(A, ws, s));
    }
    g_prep = Prepared{ws, Rp, Tp, nRp, nTp, k, m, chunk, A.agen, A.abits};
    return 0;
}

namespace {
// A frozen-first walk found at a chunk size above FF_CHUNK is restarted at FF_CHUNK (a fresh call on
// the same workspace: the carve, the preparation and every chunk's state are laid out again).  The
// restart keeps what the first attempt learned or handed out: the exact first step, the caller's
// resolved text position (EmitTarget::resolve is called once per compress) and round1_queued.
constexpr int WALK_RECHUNK = -2;
// A range walk (sccg_walk_range): the global walk from state (x0, P0) until the first index >= x_end
// (orc_walk_range's contract, compression.cpp:64-161 entered mid-way), on chunks covering
// [x0, min(x_end, |T'|)).  P0 == -1 (ungated) only at x0 == 0: the usual exact first step.  Chains,
// the frozen-first probe and the pre-queued device first step are off (accelerations whose
// bookkeeping assumes the whole target); the frozen scans stop at x_end.
struct RangeWalk {
    int64_t x0 = 0, P0 = -1, x_end = 0;
    int64_t exit_x = 0, exit_P = -1;        // out
};
struct Rechunk {
    bool on = false;                        // this is the restart
    bool resolved = false;                  // late_out->resolve was called: its output pointer
    uint8_t* out = nullptr;
    bool r1 = false;                        // late_out->round1_queued was called
    int32_t first_y = 0, first_p = 0, first_l = 0;
};

int match_and_emit_impl(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk,
                        void* ws, size_t ws_bytes, uint8_t* out, int64_t* out_len, WalkResult* res, hipStream_t s,
                        bool abs_p, const EmitTarget* late_out, bool keep_flat, Rechunk* rt, RangeWalk* rw = nullptr) {
    if (m < 0 || 2 * m + 1 > WCAP || k > KMAX || k < 1) return SCCG_E_UNSUPPORTED;
    const bool range = rw != nullptr;
    if (range && (rw->x0 < 0 || rw->P0 < -1 || (rw->P0 == -1 && rw->x0 != 0) || rw->x0 > nTp || rw->P0 >= nRp))
        return SCCG_E_UNSUPPORTED;
    const Prepared g = g_prep;   // queued by global_prepare (the caller ordered s after it)
    g_prep = Prepared{};
    const bool prepared = g.ws == ws && g.R == Rp && g.T == Tp && g.nR == nRp && g.nT == nTp && g.k == k && g.m == m &&
                          g.chunk == chunk;
    size_t used = 0;
    WalkPtrs A = make_ptrs(Rp, nRp, Tp, nTp, k, m, chunk, ws, ws_bytes, &used, prepared ? g.abits : 0);
    if (used > ws_bytes) return SCCG_E_INTERNAL;
    res->rounds = 0;
    res->chains = 0;
    res->n_matches = 0;
    const int32_t lastk = (int32_t)nTp - k;
    // a range walk's exit when it takes no match: literal steps up to min(x_end, |T'| - k + 1)
    auto literal_exit = [&](int64_t from) -> int64_t {
        const int64_t lim = rw->x_end < (int64_t)lastk + 1 ? rw->x_end : (int64_t)lastk + 1;
        return from < lim ? lim : from;
    };
    if (range) {
        const int64_t xe = rw->x_end < nTp ? rw->x_end : nTp;
        A.xlo = (int32_t)rw->x0;
        A.xhi = (int32_t)(xe > rw->x0 ? xe : rw->x0);
        A.C = (int32_t)(((int64_t)A.xhi - A.xlo + chunk - 1) / chunk);
        if (A.C < 1) A.C = 1;
        g_last_n = 0;
        if (nRp < k || lastk < 0) {   // no k-mer to probe: every step is a literal
            rw->exit_x = literal_exit(rw->x0);
            rw->exit_P = rw->P0;
            return 0;
        }
    }
    res->chunks = A.C;

    // ---- anchors -> speculative guesses for chunks 1..C-1 (queued first: they do not depend on
    //      the first step, so the GPU builds them while the host waits for it)
    const bool dbgp = getenv("SCCG_DEBUG") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!dbgp) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[phase]   walk.%-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    const bool walkable = nRp >= k && lastk >= 0;
    const unsigned gsweep = grid_for(nRp - k + 1 > 0 ? nRp - k + 1 : 1, 256 * FC_PER_T) > PRESENCE_GRID
                                ? PRESENCE_GRID : grid_for(nRp - k + 1 > 0 ? nRp - k + 1 : 1, 256 * FC_PER_T);
    if (prepared) A.agen = g.agen;
    else RC(queue_prepare(A, ws, s));

    // ---- round 1 is queued before the host knows the first step: k_walk_init<true> resolves the
    //      usual start on the device, and the round's status comes back with the first-step
    //      statistics in one readback (a host round trip less).  If the first step is not the
    //      usual one, that round is dropped and everything below runs as before.
    // (dev_nlist: the list length is the previous round tail's pending count, scal[0])
    auto queue_round = [&](int fbase_cap, bool dev_nlist) -> int {
        const int32_t* nd = dev_nlist ? A.scal : nullptr;
        PROF_LAUNCH(PROF_WALK, s, walk_kernel(A), dim3(grid_for(A.C, WWPB)), dim3(64 * WWPB), 0, s, A, (const int32_t*)A.plist,
                    A.C, nd);
        // a round that walks every chunk (round 1) carries nothing: a carry needs an unlisted successor
        if (dev_nlist) RC(launch_carry(A, s));
        hipLaunchKernelGGL(k_commit, dim3(grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256)), dim3(256), 0, s, A,
                           (const int32_t*)A.plist, A.C, nd);
        hipLaunchKernelGGL(k_list_sort, dim3(1), dim3(LS_T), 0, s, A, A.flist, (const int32_t*)(A.scal + 5), A.fbits);
        if (fbase_cap > 0) hipLaunchKernelGGL(k_frozen_scan, dim3(FZ_GRID, fbase_cap), dim3(FZ_T), 0, s, A, 0);
        SCCG_HIP(hipGetLastError());
        RC(launch_round_end(A, 0, fbase_cap, s));
        return 0;
    };
    static const bool dev_first = getenv("SCCG_HOST_FIRST_STEP") == nullptr;
    // Round 2 usually settles every chunk (round 1 speculates, round 2 confirms): with the device
    // first step it goes out right behind round 1 (its list length read on the device), followed by
    // its record text when the caller resolves the text position (late_out) -- one host readback
    // for the first step, both rounds and the text.  If round 2 left work (pending chunks, more
    // frozen chunks, escalations) that text is simply written again after the last round.
    static const bool spec_text_on = getenv("SCCG_NO_SPEC_TEXT") == nullptr;
    const bool dbg_rounds = getenv("SCCG_DEBUG") != nullptr;
    bool pre_round = false, spec_queued = false;
    int32_t rs_pre[6] = {};
    if (walkable && dev_first && !rt->on && !range && A.C > 0) {
        hipLaunchKernelGGL(k_walk_init<true>, dim3(grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256)), dim3(256), 0, s,
                           A, 0, 0);
        A.round = 1;
        RC(queue_round(FROZEN_FIRST, false));
        if (late_out && late_out->round1_queued && !rt->r1) {
            rt->r1 = true;
            RC(late_out->round1_queued(late_out->user, s));
        }
        A.round = 2;
        RC(queue_round(FROZEN_FIRST, true));
        pre_round = true;
    }

    int32_t first_y = INVALID, first_p = 0, first_l = 0;
    // ---- record text emission (k_chunk_text), queued after the rounds or speculatively (below)
    bool resolved = false, spec_text = false, text_done = false;
    int64_t spec_r[2] = {0, 0};   // total chunk matches, text bytes
    auto resolve_out = [&]() -> int {
        if (!resolved && late_out) {
            if (rt->resolved) {
                out = rt->out;
            } else {
                RC(late_out->resolve(late_out->user, &out));
                rt->resolved = true;
                rt->out = out;
            }
        }
        resolved = true;
        return 0;
    };
    // (dev_first: the first match is the device's resolution of the usual first step, see k_chunk_text)
    auto queue_text = [&](bool long_copy, bool dev_first) -> int {
        const int32_t nf = dev_first ? 2 : first_y != INVALID ? 1 : 0;
        if (A.C <= CP_MAX) {
            hipLaunchKernelGGL(k_chunk_prefix, dim3(1), dim3(1024), 0, s, A);
        } else {
            const unsigned gc = grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256);
            hipLaunchKernelGGL(k_chunk_meta, dim3(gc), dim3(256), 0, s, A);
            RC(dev_excl_max(A.cprev, A.cprev, A.C, nullptr, A.partial, s));
            RC(dev_excl_sum(A.flat_off, A.flat_off, A.C, A.scal64, A.partial, s));
            RC(set_u64(reinterpret_cast<unsigned long long*>(A.scal64 + 2), {0}, s));
        }
        const FirstMatch F{first_y, first_p, first_l, nf};
        hipLaunchKernelGGL(k_chunk_text<false>, dim3(grid_for(A.C, WPB)), dim3(SCCG_BLOCK), 0, s, A, F, (int)abs_p, out);
        RC(dev_excl_sum(A.ctext, A.ctext, A.C, A.scal64 + 1, A.partial, s));
        PROF_LAUNCH(PROF_MATCH_EMIT, s, k_chunk_text<true>, dim3(grid_for(A.C, WPB)), dim3(SCCG_BLOCK), 0, s, A, F,
                    (int)abs_p, out);
        if (long_copy) hipLaunchKernelGGL(k_long_copy, dim3(1024), dim3(256), 0, s, A, out);
        SCCG_HIP(hipGetLastError());
        return 0;
    };

    // ---- the exact first (ungated) step: first target position with any candidate
    if (walkable && range && rw->P0 >= 0) {   // (a range walk from a gated state: no first step)
    } else if (walkable && rt->on) {   // (a re-chunked restart: found by the first attempt)
        first_y = rt->first_y;
        first_p = rt->first_p;
        first_l = rt->first_l;
    } else if (walkable) {
        int32_t x0 = 0;
        unsigned long long r[9];   // fc[4..11]: first hit, first exotic, statistics of the batch's x0; fc[12]
        if (pre_round) {
            // the text of the usual first step needs (first_y, first_p, first_l) = the device's start
            // resolution: known only from this readback, so the pre-queued text uses the start that
            // k_walk_init<true> derived on the device (k_chunk_text reads it from fc)
            if (!keep_flat && !dbg_rounds && spec_text_on) {
                RC(resolve_out());
                RC(queue_text(true, true));
                spec_queued = true;
            }
            const RbItem it[3] = {{A.fc + 4, r, (int)sizeof r}, {A.scal, rs_pre, (int)sizeof rs_pre},
                                  {A.scal64, spec_r, (int)sizeof spec_r}};
            RC(dev_readback(it, 3, s));
            if (!(r[8] != 2 && r[0] == 0 && r[4] > 0)) { pre_round = false; spec_queued = false; }   // not the usual first step: redo
        } else {
            const RbItem it{A.fc + 4, r, (int)sizeof r};
            RC(dev_readback(&it, 1, s));
        }
        if (r[8] == 2) {   // the early sweep's statistics are not usable: the full first-step sweep
            const unsigned g = first_sweep_grid(A);
            hipLaunchKernelGGL(k_key0<false>, dim3(g), dim3(SCCG_BLOCK), 0, s, A, 0);
            hipLaunchKernelGGL(k_cand_reduce, dim3(1), dim3(1024), 0, s, A, (int)g, 0);
            SCCG_HIP(hipGetLastError());
            const RbItem it{A.fc + 4, r, (int)sizeof r};
            RC(dev_readback(&it, 1, s));
        }
        if (r[0] == 0 && r[4] > 0) {   // x0 = 0 has candidates (k_key0)
            first_y = 0;
            const uint64_t k0 = 1ull << 32;   // pick_key(0, -1)
            const uint64_t pk = (r[5] >= 2 && r[6]) ? r[7] : ((r[6] && k0 < r[7]) ? k0 : r[7]);
            first_p = (int32_t)(uint32_t)pk;
            first_l = (int32_t)r[4];
        }
        while (x0 <= lastk && first_y == INVALID) {
            const int32_t nb = (lastk - x0 + 1) < PB ? (lastk - x0 + 1) : PB;
            RC(set_u64(A.fc + 4, {-1, -1}, s));
            const unsigned g = gsweep;
            PROF_LAUNCH(PROF_PRESENCE, s, k_presence, dim3(g), dim3(SCCG_BLOCK), 0, s, A, x0, nb);
            hipLaunchKernelGGL(k_cand_reduce, dim3(1), dim3(1024), 0, s, A, (int)g, -1);
            SCCG_HIP(hipGetLastError());
            {
                const RbItem it{A.fc + 4, r, (int)sizeof r};
                RC(dev_readback(&it, 1, s));
            }
            if (r[0] != ~0ull && r[0] < r[1]) {
                const int32_t y = (int32_t)r[0];
                if (y == x0 && r[4] > 0) {   // statistics gathered by the same sweep
                    const uint64_t k0 = 1ull << 32;   // pick_key(0, -1)
                    const uint64_t pk = (r[5] >= 2 && r[6]) ? r[7] : ((r[6] && k0 < r[7]) ? k0 : r[7]);
                    first_y = y;
                    first_p = (int32_t)(uint32_t)pk;
                    first_l = (int32_t)r[4];
                    break;
                }
                if (A.k == A.kp) { first_y = y; break; }   // exact keys: y has a candidate
                // k > KEY_K: y's first kp bases occur in R'; the exact scan decides
                FullC f;
                RC(run_fullc(A, y, -1, &f, s));
                if (f.lmax > 0) { first_y = y; first_p = f.p; first_l = (int32_t)f.lmax; break; }
                x0 = y + 1;
                continue;
            }
            if (r[1] != ~0ull) {
                FullC f;
                RC(run_fullc(A, (int32_t)r[1], -1, &f, s));
                if (f.lmax > 0) { first_y = (int32_t)r[1]; break; }
                x0 = (int32_t)r[1] + 1;
                continue;
            }
            x0 += nb;
        }
        if (first_y != INVALID && first_l == 0) {
            FullC f;
            RC(run_fullc(A, first_y, -1, &f, s));
            first_p = f.p;
            first_l = (int32_t)f.lmax;
        }
    }
    mark("first_step");
    int32_t startX, startP;
    if (range && rw->P0 >= 0) { startX = (int32_t)rw->x0; startP = (int32_t)rw->P0; }
    else if (range && (first_y == INVALID || first_y >= rw->x_end)) {   // no match before x_end
        rw->exit_x = literal_exit(0);
        rw->exit_P = -1;
        return 0;
    } else if (first_y != INVALID) { startX = first_y + first_l; startP = first_p + first_l - 1; }
    else { startX = lastk + 1 > 0 ? lastk + 1 : 0; startP = INVALID; }

    // ---- init chunk state
    const size_t C = (size_t)A.C;
    if (!pre_round)
        hipLaunchKernelGGL(k_walk_init<false>, dim3(grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256)), dim3(256), 0, s,
                           A, startX, startP);
    SCCG_HIP(hipGetLastError());
    // Frozen-first (host first step only): when the walk from the first match finds no window hit
    // for FF_MIN_CHUNKS chunks (a stuck walk: T2T-like pairs), round 1 walks chunk 0 alone, the frozen
    // chain takes the stuck stretch, and the other chunks are speculated in round 2 (k_spec_rest) --
    // instead of speculating every chunk of the stuck stretch onto an alignment the walk never takes.
    // The probe is k_frozen_scan on a stand-in entry (chunk 0's exit = the start state), reset after.
    static const bool ff_env = getenv("SCCG_NO_FROZEN_FIRST") == nullptr;
    bool frozen_first = false;
    if (ff_env && !pre_round && !rt->on && !range && startP != INVALID && lastk >= 0 && A.C >= 2 * FF_MIN_CHUNKS) {
        RC(dev_set_i32(A.flist, 1, {0}, s));
        RC(dev_set_i32(A.exitX, 1, {startX}, s));
        RC(dev_set_i32(A.exitP, 1, {startP}, s));
        RC(dev_set_i32(A.scal + 5, 1, {1}, s));
        RC(dev_set_i32(A.fy, 1, {INT32_MAX}, s));
        hipLaunchKernelGGL(k_frozen_scan, dim3(FZ_GRID, 1), dim3(FZ_T), 0, s, A, 0);
        SCCG_HIP(hipGetLastError());
        int32_t y0 = INT32_MAX;
        {
            const RbItem it{A.fy, &y0, (int)sizeof y0};
            RC(dev_readback(&it, 1, s));
        }
        RC(dev_set_i32(A.exitX, 1, {INVALID}, s));
        RC(dev_set_i32(A.exitP, 1, {INVALID}, s));
        RC(dev_set_i32(A.scal + 5, 1, {0}, s));
        frozen_first = (int64_t)y0 >= (int64_t)FF_MIN_CHUNKS * A.S;
        if (dbgp) fprintf(stderr, "[walk] frozen-first probe: first window hit %d -> %s\n", y0, frozen_first ? "on" : "off");
        static const bool rechunk_env = getenv("SCCG_RECHUNK") != nullptr;   // opt-in (see FF_CHUNK)
        if (frozen_first && rechunk_env && A.S > FF_CHUNK) {
            rt->first_y = first_y;
            rt->first_p = first_p;
            rt->first_l = first_l;
            return WALK_RECHUNK;
        }
    }
    if (rt->on) frozen_first = true;   // (the first attempt's probe)

    if (startP != INVALID && lastk >= 0) {
        mark("anchors");
        int32_t nlist = frozen_first ? 1 : A.C;   // (k_walk_init listed chunk j at plist[j])
        const bool dbg = getenv("SCCG_DEBUG") != nullptr;
        static const bool chains_env = getenv("SCCG_NO_CHAINS") == nullptr;   // (A/B and tests)
        bool chains_on = chains_env && !range;   // off for the rest of the call after a trapped chain
        static const bool march_chains = [] { const char* e = getenv("SCCG_MARCH_CHAINS"); return e ? atoi(e) != 0 : true; }();
        int march = 0;
        int32_t prev_pend = -1;
        A.ch_settled = 0;
        // with the device first step, rounds 1 and 2 went out before the first readback
        const int64_t round0 = pre_round ? 2 : 1;
        // Rounds queued blind (SCCG_ROUND_BATCH, from round ROUND_BATCH_FROM on): once the first rounds
        // settled the bulk, the stuck / trapped targets go on for tens of rounds with few pending
        // chunks each, and a host readback per round costs as much as the round's kernels.  A
        // batch queues `batch` whole rounds back to back -- every kernel takes the pending count
        // from device memory (scal[0], written by the previous round's end; a round with nothing
        // pending is a handful of empty launches) -- and the host reads the status once, behind the
        // last.  Frozen chunks beyond the blind batch's FROZEN_FIRST, escalations and chains are
        // handled after that readback exactly as after a single round: a blind round only leaves
        // such chunks pending, so the loop's exactness argument is unchanged.
        static const int round_batch = [] { const char* e = getenv("SCCG_ROUND_BATCH"); const int v = e ? atoi(e) : ROUND_BATCH_DEFAULT; return v >= 1 && v <= 64 ? v : ROUND_BATCH_DEFAULT; }();
        int batch = 1;
        for (int64_t round = round0;; round++) {
            A.round = (int32_t)round;   // every kernel of the round gets it by value
            const bool queued = pre_round && round == round0;
            if (!queued) {
                for (int b = 0; b < batch; b++) {
                    A.round = (int32_t)(round + b);
                    const bool dev = b > 0;   // the batch's later rounds: list length on the device
                    const int32_t gl = dev ? A.C : nlist;
                    PROF_LAUNCH(PROF_WALK, s, walk_kernel(A), dim3(grid_for(gl, WWPB)), dim3(64 * WWPB), 0, s, A,
                                (const int32_t*)A.plist, gl, dev ? (const int32_t*)A.scal : (const int32_t*)nullptr);
                    SCCG_HIP(hipGetLastError());
                    if (dev || gl < A.C) RC(launch_carry(A, s));   // (every chunk listed: no carries)
                    // Commit, fill the first frozen runs and find the next round's pending chunks
                    // without waiting for the host; more frozen chunks and the rare escalated
                    // (pn2 == 0) ones are handled after the batch's one sync.
                    hipLaunchKernelGGL(k_commit, dim3(grid_for(gl, 256) > 4096 ? 4096 : grid_for(gl, 256)), dim3(256), 0, s, A,
                                       (const int32_t*)A.plist, gl, dev ? (const int32_t*)A.scal : (const int32_t*)nullptr);
                    hipLaunchKernelGGL(k_list_sort, dim3(1), dim3(LS_T), 0, s, A, A.flist, (const int32_t*)(A.scal + 5), A.fbits);
                    if (b + 1 < batch) {   // a whole round; the last one's end is queued below
                        hipLaunchKernelGGL(k_frozen_scan, dim3(FZ_GRID, FROZEN_FIRST), dim3(FZ_T), 0, s, A, 0);
                        RC(launch_round_end(A, 0, FROZEN_FIRST, s));
                    }
                }
                round += batch - 1;
                A.round = (int32_t)round;
            }
            res->rounds = round;
            auto frozen_batch = [&](int fbase, int fcap, bool init_fy) -> int {   // no-op past the list
                if (init_fy) SCCG_HIP(hipMemsetD32Async((hipDeviceptr_t)A.fy, INT32_MAX, fcap, s));
                if (fcap > 0) hipLaunchKernelGGL(k_frozen_scan, dim3(FZ_GRID, fcap), dim3(FZ_T), 0, s, A, fbase);
                SCCG_HIP(hipGetLastError());
                RC(launch_round_end(A, fbase, fcap, s));   // fills + pending
                return 0;
            };
            int32_t rs[6];
            const RbItem rs_item{A.scal, rs, (int)sizeof rs};
            if (queued) {
                for (int i = 0; i < 6; i++) rs[i] = rs_pre[i];
                spec_text = spec_queued && rs[5] <= FROZEN_FIRST && rs[1] == 0;   // nothing changes after that readback
            } else {
                RC(frozen_batch(0, FROZEN_FIRST, false));   // fy was set by k_commit
                RC(dev_readback(&rs_item, 1, s));
            }
            // A chain pays where rounds would resolve a frozen stretch hit by hit: frozen chunks still
            // turning up from round SCCG_CHAIN_ROUND (default 10) on.  (A frozen chunk in round 1 --
            // only chunk 0 is exact there, so the true walk froze at once -- starts one too, but only
            // on the host-first-step path: the default device-first path queues rounds 1 and 2
            // before its first readback and starts this loop at round 2, where round 2's frozen
            // chunks stay with the blind batches.)  Earlier frozen chunks (N gaps of aligned pairs,
            // short frozen stretches) stay with the blind batches.  Measured (start round 3 / 6 /
            // 10): synthetic chr22 2.3 / 1.7 / 1.7 ms, 20 Mb T2T-like pair 5.5 / 5.7 / 5.7 ms, 100 Mb
            // T2T-like pair 14.0 / 14.4-17.6 / 12.4 ms (23 ms without chains).
            static const int chain_round = [] { const char* e = getenv("SCCG_CHAIN_ROUND"); const int v = e ? atoi(e) : 10; return v >= 2 ? v : 10; }();
            // A march: chains are off (a trapped hand-back) and the rounds settle one or two chunks each
            // -- the frontier chunk ends frozen, its frozen scan finds the next hit a chunk on, and the
            // chunks behind it keep re-walking from entries that are not final.  A chain from the
            // frontier (the settled frozen chunk) walks those hits on the device instead.
            if (!chains_on && rs[0] > 0 && prev_pend >= 0 && rs[0] <= prev_pend && prev_pend - rs[0] <= 2) march++;
            else march = 0;
            prev_pend = rs[0];
            static const int march_rounds = [] { const char* e = getenv("SCCG_MARCH_ROUNDS"); const int v = e ? atoi(e) : MARCH_ROUNDS; return v >= 1 ? v : MARCH_ROUNDS; }();
            const bool march_chain = march_chains && chains_env && !range && !chains_on && march >= march_rounds && rs[5] > 0;
            const bool chain_now = (chains_on && rs[5] > 0 && (round == 1 || round >= chain_round)) || march_chain;
            if (chain_now) {
                A.ch_settled = march_chain ? 1 : 0;
                static const bool march_reset = [] { const char* e = getenv("SCCG_MARCH_RESET"); return e ? atoi(e) != 0 : false; }();
                if (march_chain && march_reset) march = 0;
                // a frozen chain: walk it on over the rest of the target, then the pending list again
                int gens = 0;
                bool trapped = false, started = true;
                RC(run_chain(A, s, &gens, &trapped, &started));
                static const bool keep_chains = getenv("SCCG_KEEP_CHAINS") != nullptr;   // (A/B)
                if (trapped && !keep_chains) chains_on = false;   // a trapped walk: the rounds' re-speculation resolves it
                if (started) {
                    RC(frozen_batch(0, 0, false));
                    RC(dev_readback(&rs_item, 1, s));
                    spec_text = false;   // the chain rewrote chunks after the round's text was queued
                    res->chains++;
                } else {
                    //  a march chain with no settled frozen chunk: nothing ran, so the round
                    // takes the frozen batches past the blind one as usual and the march restarts
                    march = 0;
                    if (rs[5] > FROZEN_FIRST) {
                        for (int fb = FROZEN_FIRST; fb < rs[5]; fb += FROZEN_MAX) RC(frozen_batch(fb, FROZEN_MAX, true));
                        RC(dev_readback(&rs_item, 1, s));
                    }
                }
            } else if (rs[5] > FROZEN_FIRST) {   // more frozen chunks than the blind batch covered
                for (int fb = FROZEN_FIRST; fb < rs[5]; fb += FROZEN_MAX) RC(frozen_batch(fb, FROZEN_MAX, true));
                RC(dev_readback(&rs_item, 1, s));
            }
            if (rs[1]) {
                {   // escalations: resolve on the host, resume, commit the resumed chunks
                    std::vector<int32_t> resumed;
                    RC(resolve_escalations(A, s, &resumed));
                    RC(h2d_sync(A.rlist, resumed.data(), resumed.size() * 4, s));
                    const int32_t nr = (int32_t)resumed.size();
                    RC(dev_set_i32(A.scal + 5, 1, {0}, s));   // frozen list of the resumed chunks
                    hipLaunchKernelGGL(k_commit, dim3(grid_for(nr, 256) > 4096 ? 4096 : grid_for(nr, 256)), dim3(256), 0, s, A,
                                       (const int32_t*)A.rlist, nr, (const int32_t*)nullptr);
                    hipLaunchKernelGGL(k_list_sort, dim3(1), dim3(LS_T), 0, s, A, A.flist, (const int32_t*)(A.scal + 5), A.fbits);
                    SCCG_HIP(hipGetLastError());
                }
                {
                    const RbItem it{A.scal + 5, &rs[5], (int)sizeof(int32_t)};
                    RC(dev_readback(&it, 1, s));
                }
                if (rs[5] == 0) RC(frozen_batch(0, 0, false));   // pending only
                for (int fb = 0; fb < rs[5]; fb += FROZEN_MAX) RC(frozen_batch(fb, FROZEN_MAX, fb > 0));
                RC(dev_readback(&rs_item, 1, s));
            }
            nlist = rs[0];
            static const bool round_log = getenv("SCCG_ROUND_LOG") != nullptr;   // (determinism diagnostics)
            if (round_log) {
                // (with SCCG_ROUND_LOG=2 also a digest of the chunk states, to find where two runs part)
                uint64_t hsh = 0;
                if (getenv("SCCG_ROUND_LOG")[0] == '2') {
                    std::vector<int32_t> v(C);
                    const int32_t* arrs[6] = {A.exitX, A.exitP, A.usedX, A.usedP, A.cur, A.plist};
                    for (int a = 0; a < 6; a++) {
                        const size_t nn = a == 5 ? (size_t)(rs[0] > 0 ? rs[0] : 0) : C;
                        SCCG_HIP(hipMemcpy(v.data(), arrs[a], nn * 4, hipMemcpyDeviceToHost));
                        if (a == 5) std::sort(v.begin(), v.begin() + nn);
                        for (size_t i = 0; i < nn; i++) hsh = (hsh ^ (uint32_t)v[i]) * 0x100000001b3ull + a;
                    }
                }
                fprintf(stderr, "[round] %lld pending %d esc %d frozen %d chains %lld digest %016llx\n", (long long)round, rs[0], rs[1],
                        rs[5], (long long)res->chains, (unsigned long long)hsh);
            }
            if (dbg) {
                SCCG_HIP(hipStreamSynchronize(s));
                static thread_local auto tprev = std::chrono::steady_clock::now();
                const auto tnow = std::chrono::steady_clock::now();
                fprintf(stderr, "[walk] round %lld: %d walked, %.3f ms since last mark\n", (long long)round, nlist,
                        std::chrono::duration<double, std::milli>(tnow - tprev).count());
                tprev = tnow;
            }
            static const bool dbg_all = getenv("SCCG_DEBUG_ALLROUNDS") != nullptr;
            if (dbg && (round <= 2 || dbg_all)) {   // per-chunk cost profile of the rounds' walked chunks
                constexpr size_t DS = DBG_SLOTS;
                std::vector<uint64_t> d(C * DS);
                SCCG_HIP(hipMemcpyAsync(d.data(), A.dbg, C * DS * 8, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipStreamSynchronize(s));
                std::vector<uint64_t> tk(C);
                uint64_t sum[14] = {};
                const int64_t rep = A.dbg_round > 0 ? A.dbg_round : round;   // (the round whose counters are kept)
                for (size_t j = 0; j < C; j++) {
                    const bool mine = d[j * DS + 14] == (uint64_t)rep;
                    tk[j] = mine ? d[j * DS] : 0;
                    if (mine) for (int i = 0; i < 14; i++) sum[i] += d[j * DS + i];
                }
                std::vector<uint64_t> sorted = tk;
                std::sort(sorted.begin(), sorted.end());
                {
                    int dev = 0, khz = 0;
                    (void)hipGetDevice(&dev);
                    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
                    fprintf(stderr, "[walk] wall clock rate %d kHz\n", khz);
                }
                fprintf(stderr, "[walk] r%lld chunk ticks(10ns): mean %.0f p50 %llu p90 %llu p99 %llu max %llu | totals: matches %llu "
                        "batches %llu wides %llu windows %llu cands %llu extbases %llu\n",
                        (long long)round, (double)sum[0] / C, (unsigned long long)sorted[C / 2], (unsigned long long)sorted[C * 9 / 10],
                        (unsigned long long)sorted[C * 99 / 100], (unsigned long long)sorted[C - 1],
                        (unsigned long long)sum[1], (unsigned long long)sum[2], (unsigned long long)sum[3],
                        (unsigned long long)sum[4], (unsigned long long)sum[5], (unsigned long long)sum[6]);
                {   // launch spread: when the chunks' waves started and ended, from the first start
                    uint64_t s0 = ~0ull;
                    for (size_t j = 0; j < C; j++) if (d[j * DS + 14] == (uint64_t)rep && d[j * DS + 15] < s0) s0 = d[j * DS + 15];
                    std::vector<uint64_t> st, en;
                    for (size_t j = 0; j < C; j++)
                        if (d[j * DS + 14] == (uint64_t)rep) { st.push_back(d[j * DS + 15] - s0); en.push_back(d[j * DS + 15] - s0 + d[j * DS]); }
                    if (!st.empty()) {
                        std::sort(st.begin(), st.end());
                        std::sort(en.begin(), en.end());
                        const size_t m = st.size();
                        fprintf(stderr, "[walk] r%lld %zu waves: start p50 %llu p90 %llu max %llu | end p50 %llu p90 %llu p99 %llu max %llu (10ns)\n",
                                (long long)round, m, (unsigned long long)st[m / 2], (unsigned long long)st[m * 9 / 10],
                                (unsigned long long)st[m - 1], (unsigned long long)en[m / 2], (unsigned long long)en[m * 9 / 10],
                                (unsigned long long)en[m * 99 / 100], (unsigned long long)en[m - 1]);
                    }
                }
                fprintf(stderr, "[walk] r1 step phases (10ns, summed over chunks): window %llu find %llu cand+lce %llu tail %llu "
                        "hash %llu wide %llu (wide positions %llu)\n",
                        (unsigned long long)sum[7], (unsigned long long)sum[8], (unsigned long long)sum[9], (unsigned long long)sum[10],
                        (unsigned long long)sum[11], (unsigned long long)sum[12], (unsigned long long)sum[13]);
                std::vector<size_t> idx(C);
                for (size_t j = 0; j < C; j++) idx[j] = j;
                const size_t nshow = C < 5 ? C : 5;
                std::partial_sort(idx.begin(), idx.begin() + nshow, idx.end(), [&](size_t a, size_t b) { return tk[a] > tk[b]; });
                for (size_t q = 0; q < nshow; q++) {
                    const uint64_t* e = &d[idx[q] * DS];
                    fprintf(stderr, "   slow chunk %zu: ticks %llu matches %llu batches %llu wides %llu windows %llu cands %llu ext %llu "
                            "| win %llu find %llu cand %llu tail %llu hash %llu wide %llu widepos %llu\n",
                            idx[q], (unsigned long long)e[0], (unsigned long long)e[1], (unsigned long long)e[2],
                            (unsigned long long)e[3], (unsigned long long)e[4], (unsigned long long)e[5], (unsigned long long)e[6],
                            (unsigned long long)e[7], (unsigned long long)e[8], (unsigned long long)e[9], (unsigned long long)e[10],
                            (unsigned long long)e[11], (unsigned long long)e[12], (unsigned long long)e[13]);
                }
            }
            static const int dbg_chunk = getenv("SCCG_DEBUG_CHUNK") ? atoi(getenv("SCCG_DEBUG_CHUNK")) : -1;
            if (dbg && dbg_chunk >= 0 && dbg_chunk < A.C) {   // both trajectory buffers of one chunk
                const size_t j = (size_t)dbg_chunk;
                int32_t cur = 0, cn[2] = {0, 0}, ux = 0, up = 0, ex = 0, ep = 0, sq = 0;
                SCCG_HIP(hipMemcpy(&cur, A.cur + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&cn[0], A.cnt[0] + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&cn[1], A.cnt[1] + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&ux, A.usedX + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&up, A.usedP + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&ex, A.exitX + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&ep, A.exitP + j, 4, hipMemcpyDeviceToHost));
                SCCG_HIP(hipMemcpy(&sq, A.seedq + j, 4, hipMemcpyDeviceToHost));
                fprintf(stderr, "[chunk %zu] round %lld cur=%d used=(%d,%d) exit=(%d,%d) seedq=%d\n", j, (long long)round, cur, ux,
                        up, ex, ep, sq);
                for (int b = 0; b < 2; b++) {
                    const int n = cn[b] < 80 ? cn[b] : 80;
                    std::vector<int32_t> tt(n > 0 ? n : 1), pp(tt.size()), ll(tt.size());
                    if (n > 0) {
                        SCCG_HIP(hipMemcpy(tt.data(), A.bt[b] + j * A.cap, n * 4, hipMemcpyDeviceToHost));
                        SCCG_HIP(hipMemcpy(pp.data(), A.bp[b] + j * A.cap, n * 4, hipMemcpyDeviceToHost));
                        SCCG_HIP(hipMemcpy(ll.data(), A.bl[b] + j * A.cap, n * 4, hipMemcpyDeviceToHost));
                    }
                    fprintf(stderr, "  buf%d (%d):", b, cn[b]);
                    for (int q = 0; q < n; q++) fprintf(stderr, " (%d,%d,%d)", tt[q], pp[q], ll[q]);
                    fprintf(stderr, "\n");
                }
            }
            static const int dbg_rounds = getenv("SCCG_DEBUG_ROUNDS") ? atoi(getenv("SCCG_DEBUG_ROUNDS")) : 3;
            if (dbg && (round <= dbg_rounds || round % 1000 == 0)) {
                std::vector<int32_t> g(C), ex(C), ep(C), ux(C), up(C), cur(C), c0(C), c1(C);
                SCCG_HIP(hipMemcpyAsync(g.data(), A.guess, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(ex.data(), A.exitX, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(ep.data(), A.exitP, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(ux.data(), A.usedX, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(up.data(), A.usedP, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(cur.data(), A.cur, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(c0.data(), A.cnt[0], C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipMemcpyAsync(c1.data(), A.cnt[1], C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipStreamSynchronize(s));
                size_t ginv = 0, einv = 0, settled = 0;
                for (size_t j = 0; j < C; j++) {
                    ginv += g[j] == INVALID;
                    einv += ex[j] == INVALID;
                    const int32_t px = j ? ex[j - 1] : startX, pp = j ? ep[j - 1] : startP;
                    settled += (px == ux[j] && pp == up[j]);
                }
                fprintf(stderr, "[walk] round %lld launched %d: guess INVALID %zu, exit INVALID %zu, settled %zu/%zu\n",
                        (long long)round, nlist, ginv, einv, settled, C);
                std::vector<int32_t> stt(C);
                SCCG_HIP(hipMemcpyAsync(stt.data(), A.status, C * 4, hipMemcpyDeviceToHost, s));
                SCCG_HIP(hipStreamSynchronize(s));
                int shown = 0;
                for (size_t j = 1; j < C && shown < 6; j++) {
                    if (ex[j - 1] == ux[j] && ep[j - 1] == up[j]) continue;
                    shown++;
                    fprintf(stderr, "  unsettled %zu lo=%d guess=%d used=(%d,%d) pred_exit=(%d,%d) exit=(%d,%d) st=%d cur=%d cnt=%d/%d\n",
                            j, (int)(j * A.S), g[j], ux[j], up[j], ex[j - 1], ep[j - 1], ex[j], ep[j], stt[j], cur[j], c0[j], c1[j]);
                    const int32_t b = cur[j];
                    const int32_t nshow = (b ? c1[j] : c0[j]) < 4 ? (b ? c1[j] : c0[j]) : 4;
                    std::vector<int32_t> tt(4), pp(4), ll(4);
                    SCCG_HIP(hipMemcpyAsync(tt.data(), A.bt[b] + j * A.cap, 16, hipMemcpyDeviceToHost, s));
                    SCCG_HIP(hipMemcpyAsync(pp.data(), A.bp[b] + j * A.cap, 16, hipMemcpyDeviceToHost, s));
                    SCCG_HIP(hipMemcpyAsync(ll.data(), A.bl[b] + j * A.cap, 16, hipMemcpyDeviceToHost, s));
                    SCCG_HIP(hipStreamSynchronize(s));
                    for (int q = 0; q < nshow; q++) fprintf(stderr, "      m%d (%d,%d,%d)\n", q, tt[q], pp[q], ll[q]);
                }
            }
            if (frozen_first && round == 1) {   // first speculation of every chunk still never walked
                hipLaunchKernelGGL(k_spec_rest, dim3(grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256)), dim3(256), 0, s, A);
                SCCG_HIP(hipGetLastError());
                const RbItem it{A.scal, &nlist, (int)sizeof nlist};
                RC(dev_readback(&it, 1, s));
            }
            if (round == 2 && spec_text && nlist == 0) text_done = true;
            if (!nlist) break;
            // the next iteration's batch: blind rounds once past the first ones, unless this round
            // left work only the host resolves (escalations, a chain about to start)
            batch = (round + 1 >= ROUND_BATCH_FROM && !rs[1]) ? round_batch : 1;
            if (round > 4 * (int64_t)A.C + 16) return SCCG_E_INTERNAL;
            if (late_out && late_out->abandon && late_out->abandon(late_out->user)) return WALK_ABANDONED;
        }
    }

    mark("rounds");
    const int32_t nfirst = first_y != INVALID ? 1 : 0;
    if (!keep_flat) {
        // ---- record text straight from the chunks (k_chunk_text): no flattened match list
        RC(resolve_out());   // the caller's text position is known now
        int64_t text = 0, nmc = 0;
        if (startP != INVALID && lastk >= 0) {
            if (!text_done) {   // (else round 2's speculative text, long copies included, stands)
                RC(queue_text(true, false));
                const RbItem it{A.scal64, spec_r, (int)sizeof spec_r};
                RC(dev_readback(&it, 1, s));
            }
            nmc = spec_r[0];
            text = spec_r[1];
        } else if (nTp > 0) {   // no first match: the whole target is one literal
            hipLaunchKernelGGL(k_copy, dim3(grid_for(nTp, WPB * LONG_PIECE)), dim3(SCCG_BLOCK), 0, s, Tp, nTp, out);
            SCCG_HIP(hipGetLastError());
            text = nTp;
        }
        res->n_matches = nmc + nfirst;
        g_last_n = 0;
        *out_len = text;
        mark("emit");
        return 0;
    }
    // ---- flatten: first match, then every chunk's trajectory
    hipLaunchKernelGGL(k_chunk_counts, dim3(grid_for(A.C, 256) > 4096 ? 4096 : grid_for(A.C, 256)), dim3(256), 0, s, A);
    RC(dev_excl_sum(A.flat_off, A.flat_off, A.C, A.scal64, A.partial, s));
    if (nfirst) {
        RC(dev_set_i32(A.ft, 1, {first_y}, s));
        RC(dev_set_i32(A.fp, 1, {first_p}, s));
        RC(dev_set_i32(A.fl, 1, {first_l}, s));
    }
    hipLaunchKernelGGL(k_flatten, dim3(grid_for(A.C, WPB)), dim3(SCCG_BLOCK), 0, s, A, nfirst);
    SCCG_HIP(hipGetLastError());
    int64_t nchunkm = 0;
    {
        const RbItem it{A.scal64, &nchunkm, (int)sizeof nchunkm};
        RC(dev_readback(&it, 1, s));
    }
    const int64_t nm = nchunkm + nfirst;
    res->n_matches = nm;
    g_last = A;
    g_last_n = nm;
    if (range) {   // the exit state: the last chunk's (its walk ends at the first index >= x_end)
        int32_t ex[2];
        const RbItem it[2] = {{A.exitX + (A.C - 1), &ex[0], 4}, {A.exitP + (A.C - 1), &ex[1], 4}};
        RC(dev_readback(it, 2, s));
        rw->exit_x = ex[0];
        rw->exit_P = ex[1];
        return 0;
    }

    // ---- record text: literal gap + "(dp,l)" per match, then the tail literal
    RC(resolve_out());   // the caller's text position is known now
    int64_t text = 0;
    int32_t tail_from = 0;
    if (nm > 0) {
        const unsigned g = grid_for(nm, 256) > 4096 ? 4096 : grid_for(nm, 256);
        hipLaunchKernelGGL(k_match_textlen, dim3(g), dim3(256), 0, s, A, nm, (int)abs_p);
        RC(set_u64(reinterpret_cast<unsigned long long*>(A.scal64 + 2), {0}, s));
        RC(dev_excl_sum(A.tlen, A.tlen, nm, A.scal64 + 1, A.partial, s));
        PROF_LAUNCH(PROF_MATCH_EMIT, s, k_match_textwrite, dim3(grid_for(nm, SCCG_BLOCK)), dim3(SCCG_BLOCK), 0, s, A, nm, out,
                    (int)abs_p);
        hipLaunchKernelGGL(k_long_copy, dim3(1024), dim3(256), 0, s, A, out);
        SCCG_HIP(hipGetLastError());
        int32_t lt[2];
        const RbItem it[3] = {{A.scal64 + 1, &text, (int)sizeof text}, {A.ft + nm - 1, &lt[0], 4}, {A.fl + nm - 1, &lt[1], 4}};
        RC(dev_readback(it, 3, s));
        tail_from = lt[0] + lt[1];
    }
    const int64_t tail = nTp - tail_from;
    if (tail > 0) {
        hipLaunchKernelGGL(k_copy, dim3(grid_for(tail, WPB * LONG_PIECE)), dim3(SCCG_BLOCK), 0, s, Tp + tail_from, tail,
                           out + text);
        SCCG_HIP(hipGetLastError());
    }
    *out_len = text + (tail > 0 ? tail : 0);
    mark("emit");
    return 0;
}

}  // namespace

int global_walk_range(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk, void* ws,
                      size_t ws_bytes, int64_t x0, int64_t P0, int64_t x_end, int64_t* exit_x, int64_t* exit_P,
                      WalkResult* res, hipStream_t s) {
    global_prepare_reset();
    Rechunk rt;
    RangeWalk rw;
    rw.x0 = x0; rw.P0 = P0; rw.x_end = x_end;
    int64_t tl = 0;
    const int rc = match_and_emit_impl(Rp, nRp, Tp, nTp, k, m, chunk, ws, ws_bytes, nullptr, &tl, res, s, false, nullptr,
                                       true, &rt, &rw);
    if (rc) return rc;
    *exit_x = rw.exit_x;
    *exit_P = rw.exit_P;
    return 0;
}

int global_match_and_emit(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk,
                          void* ws, size_t ws_bytes, uint8_t* out, int64_t* out_len, WalkResult* res, hipStream_t s,
                          bool abs_p, const EmitTarget* late_out, bool keep_flat) {
    Rechunk rt;
    const int rc = match_and_emit_impl(Rp, nRp, Tp, nTp, k, m, chunk, ws, ws_bytes, out, out_len, res, s, abs_p, late_out,
                                       keep_flat, &rt);
    if (rc != WALK_RECHUNK) return rc;
    if (walk_workspace_bytes(nRp, nTp, k, FF_CHUNK) > ws_bytes) return SCCG_E_INTERNAL;
    rt.on = true;
    return match_and_emit_impl(Rp, nRp, Tp, nTp, k, m, FF_CHUNK, ws, ws_bytes, out, out_len, res, s, abs_p, late_out,
                               keep_flat, &rt);
}

// a workspace buffer is about to be freed: its anchor table's generations are gone with it
void walk_forget_workspace(const void* ws) {
    std::lock_guard<std::mutex> lk(g_anchor_mu);
    g_anchor_seen.erase(ws);
}
