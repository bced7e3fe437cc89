/* synth_cli.c -- sccg_synth <hg|local|t2t> <ref_len> <tgt_len> <seed> <ref.fa> <tgt.fa> */
#include "synth.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s <hg|local|t2t> <ref_len> <tgt_len> <seed> <ref.fa> <tgt.fa>\n", argv[0]);
        return 1;
    }
    int prof = !strcmp(argv[1], "local") ? SYNTH_LOCAL : !strcmp(argv[1], "t2t") ? SYNTH_T2T : SYNTH_HG;
    char *a, *b;
    size_t na, nb;
    if (synth_pair(prof, atoll(argv[2]), atoll(argv[3]), strtoull(argv[4], NULL, 10), "chrR", "chrT",
                   &a, &na, &b, &nb)) {
        fprintf(stderr, "generation failed\n");
        return 1;
    }
    FILE* f = fopen(argv[5], "wb");
    FILE* g = fopen(argv[6], "wb");
    if (!f || !g) return 1;
    fwrite(a, 1, na, f);
    fwrite(b, 1, nb, g);
    fclose(f);
    fclose(g);
    synth_free(a);
    synth_free(b);
    return 0;
}
