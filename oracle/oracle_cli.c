/*
 * oracle_cli.c -- command-line driver of the CPU restatement (TEST INFRASTRUCTURE ONLY).
 *
 *   sccg_oracle compress   <reference.fa> <target.fa> <out_record_text>
 *   sccg_oracle decompress <record_text>  <reference.fa> <out.fa>
 *
 * Writes exactly the bytes the reference writes to compressed_genome.txt
 * (compression.cpp:329) / reconstructed_genome.fa (decompression.cpp:316-323), minus 7z.
 * Prints "mode=<local|global> switch=<seg>" and the wall time of the call to stderr.
 */
#define _POSIX_C_SOURCE 199309L
#include "sccg_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static char* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = (char*)malloc((size_t)sz + 1);
    if (!b) { fclose(f); return NULL; }
    size_t got = fread(b, 1, (size_t)sz, f);
    fclose(f);
    b[got] = 0;
    *n = got;
    return b;
}

static int spit(const char* path, const char* d, size_t n) {
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    size_t w = fwrite(d, 1, n, f);
    fclose(f);
    return w == n ? 0 : -1;
}

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc != 5 || (strcmp(argv[1], "compress") && strcmp(argv[1], "decompress"))) {
        fprintf(stderr, "usage: %s compress <ref.fa> <tgt.fa> <out.txt> | decompress <rec.txt> <ref.fa> <out.fa>\n", argv[0]);
        return 1;
    }
    size_t na, nb;
    char* a = slurp(argv[2], &na);
    char* b = slurp(argv[3], &nb);
    if (!a || !b) { fprintf(stderr, "cannot read inputs\n"); return 1; }
    char* out = NULL;
    size_t nout = 0;
    double t0 = now();
    int rc;
    if (!strcmp(argv[1], "compress")) {
        rc = orc_compress(a, na, b, nb, &out, &nout);
        fprintf(stderr, "mode=%s switch=%lld\n", orc_last_mode_global() ? "global" : "local",
                (long long)orc_last_switch_segment());
    } else {
        rc = orc_decompress(a, na, b, nb, &out, &nout);
    }
    double t1 = now();
    fprintf(stderr, "rc=%d seconds=%.6f\n", rc, t1 - t0);
    if (out && spit(argv[4], out, nout)) { fprintf(stderr, "cannot write output\n"); return 1; }
    orc_free(out);
    free(a);
    free(b);
    return rc ? 1 : 0;
}
