/*
 * abi_smoke.c — proves include/tcpcsum.h is consumable from plain C, the way
 * the reference's C host code (context.c / loop.c) would call it.
 *   ./abi_smoke        : CPU-only checks (scalar drop-ins, error paths)
 *   ./abi_smoke --gpu  : also one uniform batch on the GPU vs the scalar path
 * Exit status 0 on success.
 */
#include <arpa/inet.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tcpcsum.h"

static int fails;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

int main(int argc, char **argv) {
    int gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
    CHECK(tcpcsum_abi_version() == TCPCSUM_ABI_VERSION);
    /* SURVEY.md Appendix A KATs (from the reference's own code) */
    CHECK(tcpcsum_continue(0, "\0\0", 2) == 0xffff);
    CHECK(tcpcsum_continue(0, "\0\0\x7f", 3) == 0xff80);
    CHECK(tcpcsum_pseudo(htonl(0x0A000000), htonl(0xC0A80000), htons(1500)) == 101071);
    CHECK(tcpcsum_pseudo(htonl(0x0A000000), htonl(0xC0A80000), htons(64)) == 61130);
    CHECK(tcpcsum_pseudo(htonl(0x0A000000), htonl(0xC0A80000), 0) == 44746);
    CHECK(tcpcsum_batch_uniform_dev(NULL, 0, 0, NULL, 0, NULL, 1, NULL, NULL) == TCPCSUM_EINVAL);
    CHECK(tcpcsum_batch_uniform_dev(NULL, 0, 0, NULL, 0, NULL, 0, NULL, NULL) == TCPCSUM_OK);
    CHECK(strcmp(tcpcsum_strerror(TCPCSUM_ENODEV), "no usable gfx950 device") == 0);
    char arch[64];
    int dc = tcpcsum_device_check(arch, sizeof arch);
    printf("device_check=%d arch='%s'\n", dc, arch);
    if (gpu) {
        CHECK(dc == TCPCSUM_OK);
        enum { N = 4096, L = 1500 };
        uint8_t *h = (uint8_t *) malloc((size_t) N * L);
        uint16_t *ref = (uint16_t *) malloc(N * 2), *got = (uint16_t *) malloc(N * 2);
        uint32_t *ss = (uint32_t *) malloc(N * 4);
        srand(1);
        for (size_t i = 0; i < (size_t) N * L; ++i) h[i] = (uint8_t) rand();
        for (int i = 0; i < N; ++i) {
            ss[i] = (uint32_t) tcpcsum_pseudo(htonl(0x0A000000u | i), htonl(0xC0A80000u | (i * 7)), htons(L));
            ref[i] = tcpcsum_continue(ss[i], (const char *) h + (size_t) i * L, L);
        }
        tcpcsum_ctx_t *ctx = NULL;
        CHECK(tcpcsum_ctx_create(0, 1 << 20, &ctx) == TCPCSUM_OK);
        CHECK(tcpcsum_batch_uniform_host(ctx, h, L, L, ss, 0, got, N) == TCPCSUM_OK);
        int bad = 0;
        for (int i = 0; i < N; ++i) bad += got[i] != ref[i];
        CHECK(bad == 0);
        printf("gpu host-batch mismatches: %d / %d\n", bad, N);
        tcpcsum_ctx_destroy(ctx);
        free(h); free(ref); free(got); free(ss);
    }
    printf(fails ? "FAIL\n" : "OK\n");
    return fails ? 1 : 0;
}
