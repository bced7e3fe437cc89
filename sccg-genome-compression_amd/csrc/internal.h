// internal.h -- launchers shared between the .hip translation units and the host orchestrator.
#pragma once

#include "common.h"
#include "../../include/sccg.h"

// ---- prof.cpp: per-kernel event timing (each id brackets exactly one kernel launch) -----------
enum ProfId {
    PROF_STRIP = 0,      // k_strip_write
    PROF_RUNS,           // k_runs_write
    PROF_RUNTEXT,        // k_run_textwrite
    PROF_LOCAL14,        // k_local_all (compress) / k_local_pass<14>
    PROF_LOCAL10,        // k_local_pass<10>
    PROF_LOCAL_EMIT,     // k_seg_textwrite
    PROF_FILTER,         // k_filter_write
    PROF_ANCHOR,         // k_anchor_build
    PROF_WALK,           // k_walk
    PROF_PRESENCE,       // k_presence
    PROF_FULLC,          // k_fullc
    PROF_MATCH_EMIT,     // k_match_textwrite
    PROF_WALK_CHAIN,     // k_chain_fill (end of a frozen chain)
    PROF_DC_DECODE,      // k_tok_fill
    PROF_DC_FORMAT,      // k_format
    PROF_WALK_CARRY,     // k_walk<., true>: a round's carry launch
    PROF_COUNT
};
void prof_begin(hipStream_t s, int id);
void prof_end(hipStream_t s, int id);
#define PROF_LAUNCH(id, strm, ...)        \
    do {                                  \
        prof_begin(strm, id);             \
        hipLaunchKernelGGL(__VA_ARGS__);  \
        prof_end(strm, id);               \
    } while (0)

// ---- scan.hip ---------------------------------------------------------------------------------
#include <initializer_list>
// Blocking read of up to 8 small device values (<= 4 KiB in all) behind the work queued on s,
// through pinned host memory and a spin on a sequence number (see scan.hip).
struct RbItem {
    const void* src;   // device
    void* dst;         // host
    int bytes;
};
int dev_readback(const RbItem* items, int n, hipStream_t s);
int dev_set_i64(int64_t* p, int n, std::initializer_list<int64_t> vals, hipStream_t s);
int dev_set_i32(int32_t* p, int n, std::initializer_list<int32_t> vals, hipStream_t s);
// stream-ordered write of up to 16 bytes (copied into the kernel arguments)
int dev_put_bytes(uint8_t* p, const char* bytes, int n, hipStream_t s);
// out[0, hlen) = hdr, out[hlen] = '\n', out[total - 1] = '\n' (one launch; total >= hlen + 2)
int dev_put_frame(uint8_t* out, const uint8_t* hdr, int64_t hlen, int64_t total, hipStream_t s);
// stream-ordered dst = pre, src[0, n), post (one launch)
int dev_put_framed(uint8_t* dst, const uint8_t* src, int64_t n, char pre, char post, hipStream_t s);
int64_t scan_partials_needed(int64_t n);
int dev_excl_sum(const int64_t* in, int64_t* out, int64_t n, int64_t* d_total, int64_t* d_partial,
                 hipStream_t s);
// two independent exclusive sums of n elements in the same three launches; d_partial holds
// 2 * scan_partials_needed(n)
int dev_excl_sum2(const int64_t* in0, int64_t* out0, int64_t* d_total0, const int64_t* in1, int64_t* out1,
                  int64_t* d_total1, int64_t n, int64_t* d_partial, hipStream_t s);
int dev_excl_max(const int64_t* in, int64_t* out, int64_t n, int64_t* d_total, int64_t* d_partial,
                 hipStream_t s);

// ---- ingest.hip -------------------------------------------------------------------------------
constexpr int INGEST_TILE = 8192;  // run extraction: bytes per 256-thread tile (32 per thread)
constexpr int STRIP_TILE = 4096;   // FASTA strip: bytes per wave tile (64 per lane)
enum IngestMode { INGEST_REF = 0, INGEST_TGT = 1 };
enum FilterMode { FILTER_DROP_N_UPPER = 0, FILTER_DROP_UPPERN_ONLY = 1, FILTER_UPPER = 2 };   // all uppercase
enum RunPred { RUN_LOWER = 0, RUN_N = 1 };

struct IngestScratch {
    int64_t* tile_a;      // per tile
    int64_t* tile_b;
    int64_t* tile_fa;
    int64_t* tile_fb;
    int32_t* tile_last;
    int64_t* tile_off;
    int64_t* tile_off2;
    int32_t* tile_carry;
    void* block_sums;     // (1024 + 1) x 40 bytes
    int64_t* scalars;     // [0] header start, [1] header end, [2] out len, [3] flags
    uint16_t* keep_cache = nullptr;   // per tile 64 lanes' unkept-byte codes, or null: the write pass classifies every tile
    int32_t* keep_flag = nullptr;     // per tile (k_strip_summary)
};

// Target header: first line starting with '>' (compression.cpp:210); writes [h, he) into
// scalars[0..1] (h = n when absent).
int launch_find_header(const uint8_t* buf, int64_t n, int64_t* d_scalars, hipStream_t s);
// *res = first position >= *from_slot + 1 (0 if from_slot is null) holding byte c (mode 1) or a
// '>' that starts a line (mode 0); n if none.  *ticket_slot is scratch.
int launch_first_match(const uint8_t* buf, int64_t n, const int64_t* from_slot, int mode, uint8_t c, int64_t* res,
                       int64_t* ticket_slot, hipStream_t s);
// read_genomes_from_files (compression.cpp:193-218): compacts the kept, non-space bytes of `buf`
// into `out` (original case); *d_len = kept count; in TGT mode lines [h, he) are the header.
// d_flags (optional) gets bit0 when a kept byte is '('.  With out2, the same pass also writes the
// kept bytes through the byte filter + case map `fmode` (N erase of compression.cpp:556-557 /
// decompression.cpp:108-110) into out2, *d_len2 = their count.
// Run events the target's strip emits (its write pass, RUNS): per 4 KiB FASTA tile up to RUN_SLOT
// lowercase-run starts / exclusive ends and N-run starts / exclusive ends (output positions), the
// tile's counts (rc: 4 x 16 bits) and first / last kept byte predicates (rf: bit 0 has a kept byte,
// bits 1-2 first (lower, N), bits 3-4 last); ovf is set when a tile held more events than its slots.
constexpr int RUN_SLOT = 32;
struct RunSlots {
    int32_t* sl = nullptr;
    int32_t* el = nullptr;
    int32_t* sn = nullptr;
    int32_t* en = nullptr;
    uint64_t* rc = nullptr;
    int32_t* rf = nullptr;
    int32_t* ovf = nullptr;
};
// both run lines' run arrays (as launch_runs2) from a RUNS strip's slots: d_nruns[0..1] = counts,
// *d_ovf nonzero: a tile overflowed its slots (the caller runs launch_runs2 instead); cs, ce, bev:
// ntiles scratch each; d_nT: |T| on the device
int launch_runs_from_strip(const RunSlots& rs, int64_t ntiles, const int64_t* toff, const int64_t* d_nT, int32_t* rs_l,
                           int32_t* re_l, int32_t* rs_n, int32_t* re_n, int64_t* d_nruns, int64_t* cs, int64_t* ce,
                           int32_t* bev, int64_t* d_tot, int64_t* d_partial, hipStream_t s);
int launch_fasta_strip(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header,
                       uint8_t* out, int64_t* d_len, int32_t* d_flags, const IngestScratch& sc,
                       hipStream_t s, FilterMode fmode = FILTER_UPPER, uint8_t* out2 = nullptr,
                       int64_t* d_len2 = nullptr, const RunSlots* runs = nullptr);
// Stripped bytes [seg * SEG_L, +SEG_L) of the FASTA for each slot i (segs[i] >= 0) into
// dst[i * SEG_GATHER_B ..] from the tile offsets an earlier launch_fasta_strip of it left in
// (toff = its scratch tile_off, tcarry = tile_carry; d_len = the stripped length); and the
// unfiltered copy alone from those offsets (a pair the switch probe leaves local).
constexpr int SEG_GATHER_B = 1024;
int launch_strip_gather(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header, const int64_t* toff,
                        const int32_t* tcarry, const int64_t* d_len, const int32_t* segs, int nslots, uint8_t* dst,
                        hipStream_t s);
int launch_strip_rewrite(IngestMode mode, const uint8_t* buf, int64_t n, const int64_t* d_header, uint8_t* out,
                         const IngestScratch& sc, hipStream_t s);
// maximal runs of lowercase bytes (rs_l/re_l) and of N/n bytes (rs_n/re_n), start/end inclusive,
// in one pass; d_nruns[0..1] = their counts
int launch_runs2(const uint8_t* s_in, int64_t n, int32_t* rs_l, int32_t* re_l, int32_t* rs_n, int32_t* re_n,
                 int64_t* d_nruns, int64_t* d_cnt_l, int64_t* d_cnt_n, int64_t* d_partial, hipStream_t s);
// run line text (compression.cpp:341-368): writes it to out, *d_len = bytes
int launch_run_text(const int32_t* run_s, const int32_t* run_e, int64_t nruns, int64_t n,
                    uint8_t* out, int64_t* d_len, int64_t* d_tmp, int64_t* d_partial, hipStream_t s);

// ---- local.hip --------------------------------------------------------------------------------
constexpr int SEG_L = 1000;      // compression.cpp:375
constexpr int SEG_REC_CAP = 256; // >= 2 * (1000 / 10) + 1 records per segment
struct SegStat {
    int32_t nrec;     // records written
    int32_t nmatch;   // match records
    int32_t lit;      // literal bytes
    int32_t pass;     // 1 = k pass succeeded, 2 = k2 pass succeeded, 0 = no match record
    int32_t non_n;    // segment holds a byte other than 'N' (compression.cpp:419)
    int32_t first_p;  // segment-local p of first / last match
    int32_t last_p;
    int32_t pad;
};
// SegStat.pass of a segment the local pass proved class 0 without walking it (its records are not
// computed: launch_local_proven computes them when the pair stays local)
constexpr int32_t PASS_PROVEN = -1;
int launch_local_proven(const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int64_t iters, uint32_t* recs,
                        SegStat* stat, hipStream_t s);
// segments [seg0, seg_end) of one pass (pass 2 only touches segments pass 1 left without a match;
// pass 3: pass 1 of the PASS_PROVEN segments)
int launch_local_pass(int k, int pass, int upper, const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int64_t seg0,
                      int64_t seg_end, uint32_t* recs, SegStat* stat, hipStream_t s);
// switch FSM (compression.cpp:395-473) over segments [seg0, seg_end) from counter state *state
// (min(mismatch, 5); 6 = switched): *switch_seg = first segment where mismatch > T2, or -1
// every local segment of a compress (k = 14, then k2 = 10 without a match) and the switch point
// (|R|, |T| read from device memory, so no host sync precedes it; nseg_max bounds the grid):
// ctl = {unused 0, early-exit bound INT32_MAX, switch segment INT32_MAX (= none), 0} on
// entry; cls: per-segment classes tagged with gen (never cleared: zero-filled once, gen >= 1).
// Each segment is first tried by the class-0 proof (seg_prove; SCCG_LOCAL_PROVE=0 walks every one).
int launch_local_all(const uint8_t* R, const int64_t* d_nR, const uint8_t* T, const int64_t* d_nT, int64_t nseg_max,
                     uint32_t* recs, SegStat* stat, int32_t* cls, int32_t gen, int32_t* ctl, hipStream_t s);
// The switch-window probe (local.hip k_local_probe): classes of PROBE_PAIRS segments in runs spread
// over the pair into pout[0 .. PROBE_PAIRS) (-1 unknown) and their segment indices into
// pout[PROBE_PAIRS ..); local_probe_window finds the first window among them on the host (-1: none).
#ifndef SCCG_PROBE_RUNS
#define SCCG_PROBE_RUNS 16
#endif
constexpr int PROBE_PAIRS = SCCG_PROBE_RUNS * 8;
int local_probe_applies(int64_t nseg_max);
int launch_probe_segs(const int64_t* d_nR, const int64_t* d_nT, int32_t* segs, hipStream_t s);
int launch_segment_copy(const uint8_t* src, const int64_t* d_len, const int32_t* segs, int nslots, uint8_t* dst,
                        hipStream_t s);
int launch_local_probe(const uint8_t* gR, const int64_t* d_nR, const uint8_t* gT, const int64_t* d_nT, const int32_t* segs,
                       int32_t* pout, hipStream_t s);
int local_probe_window(const int32_t* pout);
// record text for local mode (delta-encoded, compression.cpp:406-415 + :222-304) + leftover
// (abs_p: "(p," with absolute p instead, the text before delta_encode)
int launch_local_emit(const uint8_t* T, int64_t nT, int64_t iters, const uint32_t* recs,
                      const SegStat* stat, uint8_t* out, int64_t* d_len, int64_t* d_tmp_a,
                      int64_t* d_tmp_b, int64_t* d_partial, hipStream_t s, bool abs_p = false);

// ---- walk.hip ---------------------------------------------------------------------------------
struct WalkWorkspace;  // defined in walk.hip
struct WalkResult {
    int64_t n_matches;
    int64_t rounds;
    int64_t chunks;
    int64_t chains;   // frozen chains walked by k_chain_* (rounds that had a frozen chunk)
};
size_t walk_workspace_bytes(int64_t nR, int64_t nT, int k, int chunk);
// Global pass match_sequences(R', T', 14, 100, true) (compression.cpp:561) and its record text
// (compression.cpp:564-573 + delta_encode).  `ws` is device memory of walk_workspace_bytes.
// Queues the walk's input-only work (first-step key sweep, anchor index, chunk guesses) on s with
// no host sync; a later global_match_and_emit with the same ws and inputs skips it (the caller
// orders its stream after s).
int global_prepare(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk, void* ws,
                   size_t ws_bytes, hipStream_t s);
void global_prepare_reset();   // forget a preparation that will not be used
// As soon as R' exists (before |T'| is known, tn >= |T'|): the anchor samples and the positions of
// the target's first k-mer, read from the target FASTA (d_hdr: its header range).  A later
// global_prepare on the same ws/R' only extends those positions once T' exists.  |R'| is read on
// the device from d_nRp (no host round trip); nRp_bound >= |R'| sizes the workspace and the anchor
// table (ws must hold walk_workspace_bytes(nRp_bound, tn, ...)).
// the workspace at ws is freed (sccg_ctx::get, sccg_ctx_destroy): forget its anchor-table generations
void walk_forget_workspace(const void* ws);
int global_sweep_early(const uint8_t* Rp, int64_t nRp_bound, const int64_t* d_nRp, const uint8_t* tgt_fa, int64_t tn,
                       const int64_t* d_hdr, int k, int m, int chunk, void* ws, size_t ws_bytes, hipStream_t s);
// Where the record text goes, when the caller learns it only during the walk: resolve() is called
// once, after the rounds and before the text is written, and returns the output pointer.
struct EmitTarget {
    int (*resolve)(void* user, uint8_t** out);
    void* user;
    // optional, polled after every walk round: nonzero = the walk's result is not wanted (the
    // caller's local pass found no switch), so global_match_and_emit stops with WALK_ABANDONED
    int (*abandon)(void* user) = nullptr;
    // optional, called once right after round 1 is queued on the walk's stream (the caller may
    // order other work behind it)
    int (*round1_queued)(void* user, hipStream_t s) = nullptr;
};
// global_match_and_emit's return when EmitTarget::resolve/abandon gave up on the walk (not an error)
constexpr int WALK_ABANDONED = -1;
// (abs_p: absolute p on the record line, the text before delta_encode; late_out: out is ignored
// and resolved through it; keep_flat: also keep the flat match list for global_matches, else the
// text is written straight from the chunks' trajectories)
int global_match_and_emit(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m,
                          int chunk, void* ws, size_t ws_bytes, uint8_t* out, int64_t* out_len,
                          WalkResult* res, hipStream_t s, bool abs_p = false, const EmitTarget* late_out = nullptr,
                          bool keep_flat = true);
// The global walk from state (x0, P0) until the first index >= x_end (sccg_walk_range; the
// reference's walk compression.cpp:64-161 entered mid-way): its matches stay in ws (global_matches),
// the exit state comes back.  P0 == -1 only with x0 == 0 (the ungated first step).
int global_walk_range(const uint8_t* Rp, int64_t nRp, const uint8_t* Tp, int64_t nTp, int k, int m, int chunk, void* ws,
                      size_t ws_bytes, int64_t x0, int64_t P0, int64_t x_end, int64_t* exit_x, int64_t* exit_P,
                      WalkResult* res, hipStream_t s);
// the raw match list of the last global_match_and_emit (device pointers inside ws)
int global_matches(void* ws, const int32_t** t, const int32_t** p, const int32_t** l, int64_t* n);

// ---- delta.hip --------------------------------------------------------------------------------
// delta_encode (compression.cpp:222-304) over a record line X[0, n) written with ABSOLUTE p, with
// the reference's own token scan (needed when literal bytes hold '('; see delta.hip).  On a stoi
// failure *stoi_fail is set and out = X (the reference keeps the un-delta'd text).
size_t delta_workspace_bytes(int64_t n);
int delta_encode_dev(const uint8_t* X, int64_t n, uint8_t* out, int64_t out_cap, int64_t* out_len,
                     bool* stoi_fail, void* ws, hipStream_t s);

// ---- decomp.hip: see decomp.h
