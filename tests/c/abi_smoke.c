/*
 * abi_smoke.c — proves include/tcpcsum.h is consumable from plain C, the way
 * the reference's C host code (context.c / loop.c) would call it.
 *   ./abi_smoke        : CPU-only checks (scalar drop-ins, error paths)
 *   ./abi_smoke --gpu  : also a uniform host batch and a pointer-per-packet wire
 *                        batch (INTEGRATION.md level 2) on the GPU vs the scalar path
 * Exit status 0 on success.
 */
#include <arpa/inet.h>
#include <stdint.h>
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
    CHECK(strstr(tcpcsum_build_info(), "\"product\": true") != NULL);
    printf("build: %s\n", tcpcsum_build_info());
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

        /* INTEGRATION.md level 2, pointer form: the loop's separately malloc'd
         * 32 KiB out-buffers (loop.c:180-183), each holding one packet framed as
         * context.c:169-206 frames it with check 0, filled in place at the flush */
        enum { P = 256 };
        void *pkt[P];
        uint32_t plen[P];
        const tcpcsum_tuning_t tu = {0, 0, -1, 0};
        CHECK(tcpcsum_ctx_set_tuning(ctx, &tu) == TCPCSUM_OK);
        for (int i = 0; i < P; ++i) {
            uint8_t *b = (uint8_t *) malloc(32768);
            const unsigned pay = (unsigned) (rand() % 1457), tot = 44 + pay;
            memset(b, 0, 44);
            b[0] = 0x45; b[2] = (uint8_t) (tot >> 8); b[3] = (uint8_t) tot; b[8] = 255; b[9] = 6;
            const uint32_t sa = htonl(0x7F000001u), da = htonl(0x0A000000u | (uint32_t) i);
            memcpy(b + 12, &sa, 4); memcpy(b + 16, &da, 4);
            b[32] = 6 << 4; b[33] = 0x18; b[34] = 0x20; b[40] = 3; b[41] = 3; b[42] = 5;
            for (unsigned k = 0; k < pay; ++k) b[44 + k] = (uint8_t) rand();
            pkt[i] = b;
            plen[i] = tot;
        }
        uint16_t pout[P];
        uint8_t pst[P];
        /* pass 0: default (the malloc'd packets copied through the context's
         * pinned staging, nothing page-locked); pass 1: the same packets in an
         * out-buffer pool from tcpcsum_host_alloc (INTEGRATION.md level 2: the
         * pool at loop.c:180-183), filled in place, with the blocking wait */
        uint8_t *pool = (uint8_t *) tcpcsum_host_alloc((size_t) P * 32768);
        CHECK(pool != NULL);
        void *mal[P];
        for (int i = 0; i < P; ++i) mal[i] = pkt[i];
        for (int pass = 0; pass < 2 && pool; ++pass) {
            if (pass == 1)
                for (int i = 0; i < P; ++i) {
                    memcpy(pool + (size_t) i * 32768, mal[i], 32768);
                    pkt[i] = pool + (size_t) i * 32768;
                }
            CHECK(tcpcsum_ctx_set_flags(ctx, pass ? TCPCSUM_CTX_BLOCKING_WAIT : 0u) == TCPCSUM_OK);
            CHECK(tcpcsum_ctx_set_flags(ctx, 1u) == TCPCSUM_EINVAL);   /* ABI v3's AUTO_REGISTER: gone */
            tcpcsum_ctx_stats_t st0;
            CHECK(tcpcsum_ctx_get_stats(ctx, &st0) == TCPCSUM_OK);
            CHECK(tcpcsum_ipv4_batch_ptrs_host(ctx, pkt, plen, P, TCPCSUM_IPV4_FILL, pout, pst) == TCPCSUM_OK);
            int pbad = 0;
            for (int i = 0; i < P; ++i) {
                uint8_t *b = (uint8_t *) pkt[i];
                uint16_t got, want;
                uint32_t sa, da;
                memcpy(&got, b + 36, 2);
                memset(b + 36, 0, 2);
                memcpy(&sa, b + 12, 4); memcpy(&da, b + 16, 4);
                want = tcpcsum_continue(tcpcsum_pseudo(sa, da, htons((uint16_t) (plen[i] - 20))),
                                        (const char *) b + 20, (int) plen[i] - 20);
                pbad += got != want || pout[i] != want || pst[i] != TCPCSUM_PKT_OK;
            }
            tcpcsum_ctx_stats_t st;
            CHECK(tcpcsum_ctx_get_stats(ctx, &st) == TCPCSUM_OK);
            const uint64_t staged = st.pkts_staged - st0.pkts_staged, inplace = st.pkts_in_place - st0.pkts_in_place;
            if (pass == 0) CHECK(staged == P && inplace == 0);
            else CHECK(inplace == P && staged == 0);
            CHECK(st.ns_cpu_caller > st0.ns_cpu_caller);
            CHECK(pbad == 0);
            printf("gpu pointer-batch (%s) mismatches: %d / %d (caller cpu %.1f us)\n", pass ? "in place" : "staged",
                   pbad, P, (st.ns_cpu_caller - st0.ns_cpu_caller) / 1e3);
        }
        for (int i = 0; i < P; ++i) free(mal[i]);
        tcpcsum_host_free(pool);
        tcpcsum_ctx_destroy(ctx);
        free(h); free(ref); free(got); free(ss);
    }
    printf(fails ? "FAIL\n" : "OK\n");
    return fails ? 1 : 0;
}
