/*
 * sccg_oracle.h -- CPU restatement of the SCCG reference path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (libsccg.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked byte-for-byte against the reference
 * compiled from /root/reference (oracle/_ref, `make -C oracle ref`) by
 * tests/golden/make_golden.py, whose outputs are committed as fixtures under
 * tests/golden/ and re-checked by tests/test_oracle_golden.py.
 */
#ifndef SCCG_ORACLE_H
#define SCCG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes (the reference exits/throws; the oracle reports). */
#define ORC_OK            0
#define ORC_E_ALLOC       1
#define ORC_E_DELTA_STOI  2   /* stoi threw inside delta_encode (compression.cpp:279): the
                                 reference leaves the un-delta'd file and exits 1 */
#define ORC_E_FORMAT      3   /* decompression: a missing line (decompression.cpp:68-97) */
#define ORC_E_RANGE       4   /* decompression: token beyond reference (decompression.cpp:223-229) */
#define ORC_E_PARSE       5   /* decompression: stoi/substr threw (decompression.cpp:309-311) */

/* One record of match_sequences (compression.cpp:20-24,36-179).  kind 1 = match (p already
 * includes the caller's offset, as compression.cpp:153), kind 0 = literal run of the target
 * bytes St[t, t+l). */
typedef struct {
    int32_t kind;
    int32_t p;
    int32_t l;
    int64_t t;
} orc_rec;

/* compression.cpp:36 match_sequences(Sr, St, k, m, global, offset). */
int orc_match(const char* sr, int64_t nr, const char* st, int64_t nt, int k, int m, int global,
              int64_t offset, orc_rec** recs, int64_t* nrec);

/* compression.cpp:320-582 compress_genome up to (excluding) the 7z call: the exact bytes of
 * <out>/compressed_genome.txt.  On ORC_E_DELTA_STOI *out holds the un-delta'd text. */
/* The global walk (match_sequences with global = true) from state (index x0, prev_match_end P0)
 * until index >= x_end: match records only (literals are the gaps) and the exit state. */
int orc_walk_range(const char* sr, int64_t nr, const char* st, int64_t nt, int k, int m, int64_t x0, int64_t P0,
                   int64_t x_end, orc_rec** recs, int64_t* nrec, int64_t* exit_x, int64_t* exit_P);

int orc_compress(const char* ref_fa, size_t ref_len, const char* tgt_fa, size_t tgt_len,
                 char** out, size_t* out_len);

/* compress_genome's constants (compression.cpp:373-379).  orc_params_default gives the
 * reference's values (orc_compress); other values are the library's NON-PARITY overrides
 * (sccg_params in include/sccg.h): the same algorithm with other constants, which the reference
 * cannot run.  local = 0 runs the global pass (:484-574) alone. */
typedef struct {
    int k, k2, L, m;
    float T1;
    int T2, local;
} orc_params;
void orc_params_default(orc_params* p);
int orc_compress_params(const orc_params* p, const char* ref_fa, size_t ref_len, const char* tgt_fa,
                        size_t tgt_len, char** out, size_t* out_len);

/* Diagnostics of the last orc_compress in this thread: 1 if it switched to global mode,
 * and the segment index at which it switched (-1 if it stayed local). */
int orc_last_mode_global(void);
int64_t orc_last_switch_segment(void);

/* decompression.cpp:21-114 + 117-279 + 316-323 after the 7z step: the exact bytes of
 * <out>/reconstructed_genome.fa from the record text and the reference FASTA. */
int orc_decompress(const char* rec, size_t rec_len, const char* ref_fa, size_t ref_len,
                   char** out, size_t* out_len);

void orc_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
