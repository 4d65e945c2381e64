/*
 * examples/krum_cli.c -- a plain C caller of libbk.so through include/bk.h only
 * (no Python, no torch): the call sequence of the cgo shim go/bk/krum_bk.go,
 * i.e. of KRUMValidator.getTopKRUMIndex (DistSys/krum.go:100-166):
 *
 *   bk_create -> bk_check_args -> bk_stage_alloc (C-owned pinned staging) ->
 *   pack rows -> bk_multikrum(BK_HOST_PINNED) -> selected indices ->
 *   bk_selection_margin (near-tie log) -> bk_destroy
 *
 *   krum_cli <file> <n> <d> <f>     file: n*d little-endian float64, row-major
 *
 * Prints "m=<m>" and then the m selected indices (ascending), one per line,
 * and the selection margin on stderr;
 * on any error prints bk_last_error() and exits 1 (the shim rejects every
 * update in that case).  Built by __graft_entry__.build() with gcc.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bk.h"

int main(int argc, char **argv)
{
    if (argc != 5) {
        fprintf(stderr, "usage: %s <file> <n> <d> <f>\n", argv[0]);
        return 2;
    }
    const int64_t n = atoll(argv[2]), d = atoll(argv[3]), f = atoll(argv[4]);
    if (bk_check_args(n, d, f) != BK_OK) {
        fprintf(stderr, "krum_cli: %s\n", bk_last_error());
        return 1;
    }
    bk_ctx *ctx = NULL;
    if (bk_create(&ctx, 0) != BK_OK) {
        fprintf(stderr, "krum_cli: bk_create: %s\n", bk_last_error());
        return 1;
    }
    void *stage = NULL;
    const int64_t bytes = n * d * (int64_t)sizeof(double);
    int rc = 1;
    int64_t *sel = NULL;
    FILE *fp = NULL;
    if (bk_stage_alloc(ctx, bytes, &stage) != BK_OK) {
        fprintf(stderr, "krum_cli: bk_stage_alloc: %s\n", bk_last_error());
        goto out;
    }
    fp = fopen(argv[1], "rb");
    if (!fp || fread(stage, 1, (size_t)bytes, fp) != (size_t)bytes) {
        fprintf(stderr, "krum_cli: cannot read %lld bytes from %s\n", (long long)bytes, argv[1]);
        goto out;
    }
    sel = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n - f));
    int64_t m = 0;
    if (!sel || bk_multikrum(ctx, stage, BK_HOST_PINNED, BK_F64, n, d, d, f, sel, &m, NULL,
                             NULL) != BK_OK) {
        fprintf(stderr, "krum_cli: bk_multikrum: %s\n", bk_last_error());
        goto out;
    }
    printf("m=%lld\n", (long long)m);
    for (int64_t i = 0; i < m; ++i) printf("%lld\n", (long long)sel[i]);
    /* the shim's near-tie log (bk_selection_margin): stderr, stdout stays the set */
    double gap = 0, bound = 0;
    int near = 0;
    if (bk_selection_margin(ctx, &gap, &bound, &near) != BK_OK) {
        fprintf(stderr, "krum_cli: bk_selection_margin: %s\n", bk_last_error());
        goto out;
    }
    fprintf(stderr, "margin: gap=%.17g err_bound=%.17g near_tie=%d\n", gap, bound, near);
    rc = 0;
out:
    if (fp) fclose(fp);
    free(sel);
    if (stage) bk_stage_free(ctx, stage);
    bk_destroy(ctx);
    return rc;
}
