/*
 * sccg.h -- C ABI of the MI355X-native SCCG hot path (libsccg.so).
 *
 * The reference (Jan-Celin/SCCG-genome-compression) has no library or FFI: its drop-in boundary
 * is the two command lines plus the record-file format.  This header is the
 * seam a host program binds to; the repository's `compression` / `decompression` executables are
 * thin CLIs over it with the reference's argv, output paths, 7z calls and exit codes.
 *
 * Entry point                         replaces (reference file:line)
 * ----------------------------------  -------------------------------------------------------------
 * sccg_compress / _device             compress_genome up to the 7z call  compression.cpp:320-580
 * sccg_compress_files                 the same from FASTA files to the   compression.cpp:181-220,
 *                                     record file                         :320-331
 *   (_ex: with parameter overrides      of its constants                   compression.cpp:373-379)
 *                                     (read_genomes_from_files :181-220, lowercase/N run lines
 *                                     :341-368/:495-555, local loop :372-481, global pass
 *                                     :484-574, delta_encode :222-304)
 * sccg_match                          match_sequences                    compression.cpp:36-179
 * sccg_walk_range / _device           its global walk from a state        compression.cpp:64-161
 *                                     (one chromosome split across GPUs)
 * sccg_reconstruct / _device          decompress_genome after 7z +       decompression.cpp:43-114,
 *                                     reconstruct_genome + file body     :117-279, :316-323
 *
 * Conventions: status ints (0 = OK); the library never calls exit(); host buffers it returns are
 * malloc'ed and released with sccg_buf_free.  One context per GPU; a context is not re-entrant;
 * contexts on different GPUs may be driven from different host threads.  Every compute path runs
 * on the GPU -- there is no CPU fallback; without a usable device sccg_ctx_create fails.
 */
#ifndef SCCG_H
#define SCCG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCCG_OK             0
#define SCCG_E_INVALID      1  /* bad argument */
#define SCCG_E_HIP          2  /* HIP runtime error (message in sccg_last_error) */
#define SCCG_E_NOMEM        3  /* device or host allocation failed */
#define SCCG_E_DELTA_STOI   4  /* delta_encode's stoi would throw (compression.cpp:279): the
                                  reference then leaves the un-delta'd text and exits 1; the text
                                  returned is that un-delta'd text */
#define SCCG_E_FORMAT       5  /* record file misses a line (decompression.cpp:68-97) */
#define SCCG_E_RANGE        6  /* token beyond the reference (decompression.cpp:223-229) */
#define SCCG_E_PARSE        7  /* malformed run line / token (decompression.cpp:309-311) */
#define SCCG_E_UNSUPPORTED  8  /* shape outside what sccg_match accepts (see below) */
#define SCCG_E_INTERNAL     9  /* internal consistency check failed */
#define SCCG_E_OPEN_REF    10  /* reference FASTA cannot be opened / read (compression.cpp:187-191) */
#define SCCG_E_OPEN_TGT    11  /* target FASTA cannot be opened / read (compression.cpp:202-206) */
#define SCCG_E_WRITE       12  /* the record file cannot be written (compression.cpp:329-331) */

typedef struct sccg_ctx sccg_ctx;

typedef struct {
    char* data;
    size_t len;
} sccg_buf;

/* match_sequences' vector<Position> as SoA (compression.cpp:20-24): kind 1 = match (pos
 * includes the offset, :153), kind 0 = literal run St[t, t+len). */
typedef struct {
    uint8_t* kind;
    int32_t* pos;
    int32_t* len;
    int64_t* t;
    int64_t n;
} sccg_records;

typedef struct {
    int mode_global;          /* 1 when the local loop switched (compression.cpp:462-473) */
    int64_t switch_segment;   /* last segment of a switch window (compression.cpp:417-473), -1 if it
                                 stayed local: the reference's switch segment (the first window)
                                 with SCCG_OPT_EXACT_SWITCH, otherwise the first window the mode
                                 probe found (>= it; the record file is the same either way) */
    int64_t target_bases;     /* |T| after whitespace strip (compression.cpp:218) */
    int64_t reference_bases;  /* |R| */
    int64_t n_matches;        /* (p,l) tokens on the record line */
    int64_t literal_bases;    /* literal bytes on the record line */
    int64_t walk_rounds;      /* global walk: speculative + fix-up rounds */
    int64_t walk_chunks;      /* global walk: chunks */
    int64_t record_bytes;     /* length of the whole compressed_genome.txt */
    int64_t walk_chains;      /* global walk: frozen chains resolved by the chain kernels */
    int64_t walk_reference_bases; /* |R'|: the reference with every 'N' erased (compression.cpp:556) */
} sccg_stats;

int sccg_ctx_create(int device, sccg_ctx** out);
void sccg_ctx_destroy(sccg_ctx* ctx);
const char* sccg_last_error(const sccg_ctx* ctx);
int sccg_last_stats(const sccg_ctx* ctx, sccg_stats* out);

/* Context options (sccg_ctx_set_option; SCCG_E_INVALID for an unknown option):
 *   SCCG_OPT_EXACT_SWITCH  0 (default): the local/global mode is decided from ANY switch window
 *                          (a few probed runs of segments first), which is enough for the record
 *                          file (compression.cpp:462-473 truncates it and the global pass
 *                          regenerates it); 1: the in-order pass finds the first window, so
 *                          sccg_stats.switch_segment is the reference's switch segment. */
#define SCCG_OPT_EXACT_SWITCH 1
int sccg_ctx_set_option(sccg_ctx* ctx, int option, int64_t value);

/* Whole-file compression up to (excluding) 7z: returns the exact bytes of
 * <out>/compressed_genome.txt for the given reference/target FASTA file contents. */
int sccg_compress(sccg_ctx* ctx, const char* ref_fa, size_t ref_len, const char* tgt_fa,
                  size_t tgt_len, sccg_buf* out_text);

/* Same, HBM-resident: inputs are device pointers, the text is written to d_out (capacity
 * out_cap bytes; sccg_compress_bound gives a safe capacity) and *out_len is set.  `stream` is a
 * hipStream_t (NULL = the context's own stream).  Synchronises before returning. */
int sccg_compress_device(sccg_ctx* ctx, const void* d_ref_fa, size_t ref_len, const void* d_tgt_fa,
                         size_t tgt_len, void* d_out, size_t out_cap, size_t* out_len, void* stream);
size_t sccg_compress_bound(size_t ref_len, size_t tgt_len);

/* compress_genome's algorithm parameters (compression.cpp:373-379, hard-coded there).
 * sccg_params_default() gives the reference's values, with which sccg_compress_ex is
 * sccg_compress.  Other values are NON-PARITY overrides: the reference cannot
 * run them, so their output is pinned against the parameterised CPU oracle only.  Accepted:
 *   local = 1 (start with the local segment controller, :378): k, k2, L, T1, T2 at the reference's
 *             values (the local kernels are built for them), 0 <= m <= 127;
 *   local = 0 (straight to the global pass, as the reference with `local = false`): 1 <= k <= 32,
 *             0 <= m <= 127 (k2, L, T1, T2 unused).
 * Others: SCCG_E_UNSUPPORTED. */
typedef struct {
    int32_t k;       /* 14   primary k-mer length: local pass 1 and the global walk */
    int32_t k2;      /* 10   local pass 2 */
    int32_t L;       /* 1000 segment length */
    int32_t m;       /* 100  global range gate |p - prev_match_end| <= m */
    float T1;        /* 0.5  segment mismatch-ratio threshold */
    int32_t T2;      /* 4    bad segments in a row before the switch to global */
    int32_t local;   /* 1    start with the local controller */
} sccg_params;

void sccg_params_default(sccg_params* p);
int sccg_compress_ex(sccg_ctx* ctx, const sccg_params* params, const char* ref_fa, size_t ref_len,
                     const char* tgt_fa, size_t tgt_len, sccg_buf* out_text);
int sccg_compress_device_ex(sccg_ctx* ctx, const sccg_params* params, const void* d_ref_fa,
                            size_t ref_len, const void* d_tgt_fa, size_t tgt_len, void* d_out,
                            size_t out_cap, size_t* out_len, void* stream);

/* Files in, record file out (compression.cpp:320-580 up to, excluding, the 7z call): reads both
 * FASTA files (host threads, pinned staging, the copies to HBM overlapped with the reading and the
 * reference's GPU work), compresses on the GPU and writes `out_path` (the bytes sccg_compress
 * returns).  params NULL = the reference's constants.  *out_len (optional) = bytes written.
 * SCCG_E_OPEN_REF / _OPEN_TGT when an input cannot be opened (nothing written), SCCG_E_WRITE when
 * the output cannot; SCCG_E_DELTA_STOI writes the un-delta'd text as the reference does. */
int sccg_compress_files(sccg_ctx* ctx, const sccg_params* params, const char* ref_path, const char* tgt_path,
                        const char* out_path, size_t* out_len);

/* match_sequences(Sr, St, k, m, global, offset) on already-uppercased byte strings.  Accepted
 * shapes: global == 0 with |Sr| <= 1000 and |St| <= 1000 (the local-segment kernel), or
 * global == 1 with 0 <= m <= 127 and 1 <= k <= 32 (the windowed global walk).  Others:
 * SCCG_E_UNSUPPORTED. */
int sccg_match(sccg_ctx* ctx, const uint8_t* sr, size_t nr, const uint8_t* st, size_t nt, int k,
               int m, int global, int64_t offset, sccg_records* out);
void sccg_records_free(sccg_records* r);

/* The global walk of match_sequences(Sr, St, k, m, true) (compression.cpp:64-161) entered at state
 * (index = x0, prev_match_end = P0) and run until the first state with index >= x_end (or until
 * index > |St| - k): its match records (kind 1, pos = p, len = l, t = target index; the literals are
 * the gaps) and that exit state, exit_state[0] = index, exit_state[1] = prev_match_end.  This is the
 * engine of one chromosome's walk split across GPUs (multigpu.split_walk):
 * two walks that reach the same state coincide afterwards.  Sr, St: N-erased, uppercased sequences
 * (R', T' of compression.cpp:556-557).  P0 == -1 (the ungated first step) only with x0 == 0;
 * 0 <= m <= 127, 1 <= k <= 32.  The _device form takes device pointers (stream: hipStream_t or
 * NULL); both return host records (sccg_records_free). */
int sccg_walk_range(sccg_ctx* ctx, const uint8_t* sr, size_t nr, const uint8_t* st, size_t nt, int k, int m,
                    int64_t x0, int64_t P0, int64_t x_end, sccg_records* out, int64_t* exit_state);
int sccg_walk_range_device(sccg_ctx* ctx, const void* d_ref, size_t nr, const void* d_tgt, size_t nt, int k,
                           int m, int64_t x0, int64_t P0, int64_t x_end, sccg_records* out, int64_t* exit_state,
                           void* stream);

/* Decompression after 7z: record text (contents of the extracted compressed_genome.txt) +
 * reference FASTA -> exact bytes of <out>/reconstructed_genome.fa. */
int sccg_reconstruct(sccg_ctx* ctx, const char* ref_fa, size_t ref_len, const char* rec_text,
                     size_t rec_len, sccg_buf* out_fa);
/* HBM-resident form.  With d_out == NULL only *out_len (the exact output size) is computed;
 * with out_cap too small it returns SCCG_E_NOMEM and sets *out_len to the size needed. */
int sccg_reconstruct_device(sccg_ctx* ctx, const void* d_ref_fa, size_t ref_len, const void* d_rec,
                            size_t rec_len, void* d_out, size_t out_cap, size_t* out_len, void* stream);

void sccg_buf_free(sccg_buf* b);

/* Per-kernel device timing with HIP events recorded on the launching stream (process-wide).
 * sccg_profile(ctx, 1) resets and enables it for every family, 0 disables it (enable > 1: a bit
 * mask as below, kept for old callers -- it cannot select family 0 alone).  sccg_profile_mask
 * resets and enables it for the families of `mask` (bit i = sccg_profile_name(i); 0 disables).
 * sccg_profile_get returns the summed duration and launch count of one kernel family by name
 * (sccg_profile_name(i), i = 0.. until NULL). */
int sccg_profile(sccg_ctx* ctx, int enable);
int sccg_profile_mask(sccg_ctx* ctx, uint32_t mask);
int sccg_profile_get(sccg_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches);
const char* sccg_profile_name(int i);

#ifdef __cplusplus
}
#endif
#endif
