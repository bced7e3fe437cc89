// decomp.h -- launchers of decomp.hip (reconstruction), driven by sccg_api.cpp.
#pragma once
#include "internal.h"

struct DcRuns {
    int32_t* start;   // run starts (ascending, disjoint)
    int32_t* len;     // run lengths
    int64_t* cum;     // exclusive prefix of len
    int64_t n;        // runs
    int64_t total;    // sum of len
};

// Token table of the fused reconstruction (decomp.hip k_tok_emit): entry 0 a sentinel, entry 1 + j
// token j of the record line (decoded offset, absolute reference position, length, record offset
// after its ')').
struct DcTokTab {
    int64_t *o, *p, *l, *r;
};
struct DcTokBuf {
    DcTokTab tab;      // capacity dc_tok_cap(n) entries each
    int64_t* btok;     // >= n / 64 + 2: tokens per 64-byte block
    int64_t* btoff;    // >= n / 64 + 2: their exclusive prefix
    int64_t* d_ntok;   // tokens of the line (entries 1..*d_ntok)
};
int64_t dc_tok_cap(int64_t n);
// what the fused formatter reads: the token table, the record line, R' and |R'| (device)
struct DcFmtSrc {
    DcTokTab tk;
    const int64_t* d_ntok;
    const uint8_t* rec;
    int64_t nrec;
    const uint8_t* R;
    const int64_t* d_nref;
};

// every '\n' of the record text, unordered: d_buf[0] = their count, d_buf[1, 1 + DC_NL_CAP) the
// first DC_NL_CAP found (one pass; the caller sorts them, or uses dc_find_lines when there are more)
constexpr int DC_NL_CAP = 32;
// (d_err, if given, is zeroed in the same stream-ordered launch as the count)
int dc_newlines(const uint8_t* d_rec, int64_t n, int64_t* d_buf, hipStream_t s, int32_t* d_err = nullptr);
// positions of the first four '\n' of the record text (n when absent) -> d_nl[0..3]
int dc_find_lines(const uint8_t* d_rec, int64_t n, int64_t* d_nl, hipStream_t s);
// exclusive max-scan of parenthesis positions: d_lp[i] = last '(' or ')' strictly before i
// (negative when none)
int dc_last_paren(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_partial, hipStream_t s);
// parse a lowercase / N run line (decompression.cpp:126-207) into r (arrays pre-allocated with
// capacity dc_run_cap(n)); d_err bit0 set on text outside the grammar.  No host wait: d_count[0]
// = runs, d_count[1] = total run length stay on the device (the caller reads them into r->n /
// r->total); d_lp, d_flag, d_dlt hold >= max(n, dc_run_cap(n)) + 1 entries.
int64_t dc_run_cap(int64_t n);
int dc_parse_runs(const uint8_t* d_s, int64_t n, DcRuns* r, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt,
                  int64_t* d_partial, int32_t* d_err, int64_t* d_count, hipStream_t s);
// both run lines (line 0 -> r0 / d_count0, line 1 -> r1 / d_count1) in one launch set when both take
// the tiled parser (d_flag and d_dlt then hold their tile summaries), else one after the other
int dc_parse_runs2(const uint8_t* s0, int64_t n0, DcRuns* r0, int64_t* d_count0, const uint8_t* s1, int64_t n1, DcRuns* r1,
                   int64_t* d_count1, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt, int64_t* d_partial, int32_t* d_err,
                   hipStream_t s);
// d_err bit2: the last N run (count d_ncnt[0]) ends past the decoded length *d_D + N count d_ncnt[1]
int dc_n_check(const DcRuns& nr, const int64_t* d_ncnt, const int64_t* d_D, int32_t* d_err, hipStream_t s);
// record line: per-byte output contribution / token deltas, output offsets, absolute p, range
// check against *d_nref (d_err bit1 = token beyond the reference; the check waits for nref_ready
// when given); *d_total = decoded length
int dc_decode_prepare(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_contrib, int64_t* d_dlt, int64_t* d_off,
                      int64_t* d_dsum, const int64_t* d_nref, hipEvent_t nref_ready, int64_t* d_partial, int32_t* d_err,
                      int64_t* d_total, hipStream_t s, const DcTokBuf* tk = nullptr);
// fused path (tk given to dc_decode_prepare): d_err bit 2 for tokens beyond *d_nref
int dc_tok_range(const DcTokBuf& tk, int64_t cap, const int64_t* d_nref, int32_t* d_err, hipStream_t s);
// true: the reconstruction expands tokens inside the formatter (no decoded buffer); opt-in with
// SCCG_DC_FUSED=1 (A/B runs), the fill + format path otherwise
bool dc_fused();
// (tiled path, dc_tok_tiled(): the range check against *d_nref happens here, d_err bit 2)
// the tiled path's range check alone (k_tok_fill2 without writing): d_err bit 2
int dc_tok_range_tiled(const uint8_t* d_s, int64_t n, const int64_t* d_lp, const int64_t* d_off, const int64_t* d_dsum,
                       const int64_t* d_nref, int32_t* d_err, hipStream_t s);
int dc_decode_fill(const uint8_t* d_s, int64_t n, const int64_t* d_lp, const int64_t* d_off, const int64_t* d_dsum,
                   const int64_t* d_dlt, const int64_t* d_contrib, const uint8_t* d_R, uint8_t* d_dec, hipStream_t s,
                   const int64_t* d_nref, int32_t* d_err, int64_t dcap = INT64_MAX);
// true: the record line takes the per-block path (its range errors are known only after the fill)
bool dc_tok_tiled();
// N insertion + lowercase + 50-column wrap of nres result bytes into d_out (no final '\n');
// d_span: scratch of dc_format_span_words(nres) int64 (per-span run indices)
int64_t dc_format_span_words(int64_t nres);
// With fz (fused path) d_dec is unused: the decoded bytes come from fz's token table; the stream
// waits for wait_before (the reference strip) between the block index and the formatter.
// index_ready: dc_format_index already wrote the block index into d_span (on another stream,
// ordered before wait_before).
int dc_format(const uint8_t* d_dec, int64_t nres, const DcRuns& nr, const DcRuns& lr, int64_t* d_span, uint8_t* d_out,
              hipStream_t s, const DcFmtSrc* fz = nullptr, hipEvent_t wait_before = nullptr, bool index_ready = false);
// The unfused formatter's block index alone (it needs the run lists, not the decoded bytes, so it
// can run beside the token fill); returns false (nothing launched) where dc_format builds its own.
bool dc_format_index(int64_t nres, const DcRuns& nr, const DcRuns& lr, int64_t* d_span, uint8_t* d_out, hipStream_t s,
                     int* rc);
