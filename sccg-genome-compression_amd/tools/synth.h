/*
 * synth.h -- deterministic synthetic chromosome-pair generator.
 *
 * The reference's only data (hg18/hg19 chr19, .MISSING_LARGE_BLOBS) is not available offline,
 * so tests and bench.py use reference/target FASTA pairs generated here from a seed.
 * Profiles:
 *   SYNTH_HG     uniform background, 300-bp repeat family (10 % cover, 10 % divergent, poly-A
 *                tails), 45 % soft-masking, 10 kb terminal N gaps + a centromeric gap; target =
 *                reference + 1e-3 SNPs + 1e-4 indels (1-20 bp) + kb-scale insertions (they force
 *                the global switch, as compression.cpp:462-473 does on real pairs).
 *   SYNTH_LOCAL  as SYNTH_HG with SNPs only (the walk stays in local mode).
 *   SYNTH_T2T    divergent: 171-bp tandem arrays, 1e-2 SNPs, >100-bp deletions every ~100 kb,
 *                reference has N gaps, target none (drives the literal-heavy global path).
 */
#ifndef SCCG_SYNTH_H
#define SCCG_SYNTH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SYNTH_HG = 0, SYNTH_LOCAL = 1, SYNTH_T2T = 2 };

/* Generates both FASTA texts (">name\n" + 50-column lines).  Buffers are malloc'ed; free them
 * with synth_free.  Returns 0 on success. */
int synth_pair(int profile, int64_t ref_len, int64_t tgt_len, uint64_t seed, const char* ref_name,
               const char* tgt_name, char** ref_fa, size_t* ref_n, char** tgt_fa, size_t* tgt_n);

void synth_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
