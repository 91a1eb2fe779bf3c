/* svc_lat.c -- per-call latency of small host-memory batches from plain C
 * (no interpreter in the timed calls): the resident service
 * (qhuff_svc_encode / _decode), the host batch path on a context without a
 * service (qhuff_*_batch_host: launch + copies + synchronisation per call),
 * and the per-string entry point qhuff_enc_enc_str with and without a
 * service attached.  Prints one JSON object.
 *
 * build: gcc -O2 -std=c11 -pthread -I include tools/svc_lat.c \
 *            -o tools/svc_lat -L ls-qpack_amd -lqhuff \
 *            -Wl,-rpath,'$ORIGIN/../ls-qpack_amd' 
 * usage: tools/svc_lat [calls] */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "qhuff.h"

static double
now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int
cmp_d(const void *a, const void *b)
{
    const double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

struct stat3
{
    double p50, p90, p99;
};

static struct stat3
stats(double *t, int k)
{
    qsort(t, k, sizeof(double), cmp_d);
    struct stat3 s = {t[k / 2], t[(int) (k * 0.9)], t[(int) (k * 0.99)]};
    return s;
}

static void
put(const char *name, struct stat3 s, int last)
{
    printf("\"%s\": {\"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f}%s", name,
           s.p50, s.p90, s.p99, last ? "" : ", ");
}

#define CHK(x)                                                               \
    do {                                                                     \
        int r_ = (x);                                                        \
        if (r_) {                                                            \
            fprintf(stderr, "%s: %d\n", #x, r_);                             \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

/* throughput: T threads each encoding header blocks through the service */
struct tp_arg
{
    qhuff_svc *svc;
    const uint8_t *data;
    const uint32_t *off;
    uint32_t n;
    double secs;
    long calls;
};

static void *
tp_worker(void *p)
{
    struct tp_arg *a = p;
    uint8_t out[8192];
    uint32_t oo[65];
    const double t0 = now_us();
    long k = 0;
    while (now_us() - t0 < a->secs * 1e6)
    {
        CHK(qhuff_svc_encode(a->svc, a->data, a->off, a->n, 0, out, oo));
        ++k;
    }
    a->calls = k;
    return NULL;
}

int
main(int argc, char **argv)
{
    const int calls = argc > 1 ? atoi(argv[1]) : 5000;
    const uint32_t ns[] = {1, 20, 64, 256, 1024};
    double *t = malloc(sizeof(double) * calls);
    qhuff_ctx *plain, *sc;
    qhuff_svc *svc;
    CHK(qhuff_open(0, &plain));
    CHK(qhuff_open(0, &sc));
    CHK(qhuff_svc_open(sc, 0, 0, &svc));
    printf("{\"calls\": %d, \"cases\": {", calls);
    for (unsigned c = 0; c < sizeof(ns) / sizeof(ns[0]); ++c)
    {
        const uint32_t n = ns[c];
        uint8_t *data = malloc(64 * n + 64);
        uint32_t *off = malloc(4 * (n + 1));
        const uint64_t raw = qhuff_synth_batch(1000 + n, n, 8, 64,
                                               (const uint8_t *) "abcdefghijklmnopqrstuvwxyz"
                                               "0123456789-_.", 39, data, off);
        const uint64_t eb = qhuff_encode_bound(raw, n, 0);
        uint8_t *enc = malloc(eb), *dec = malloc(raw + 64), *st = malloc(n);
        uint32_t *eoff = malloc(4 * (n + 1)), *doff = malloc(4 * (n + 1));
        CHK(qhuff_encode_batch_host(plain, data, off, n, 0, enc, eoff));
        uint8_t *huff = malloc(eoff[n] + 16);
        uint32_t *hoff = malloc(4 * (n + 1));
        memcpy(huff, enc, eoff[n]);
        memcpy(hoff, eoff, 4 * (n + 1));
        printf("%s\"%u\": {\"raw_bytes\": %llu, \"huff_bytes\": %u, ",
               c ? ", " : "", n, (unsigned long long) raw, hoff[n]);
        for (int p = 0; p < 4; ++p)
        {
            const int is_dec = p & 1, is_svc = p < 2;
            for (int i = -50; i < calls; ++i)
            {
                const double a = now_us();
                if (is_svc && !is_dec)
                    CHK(qhuff_svc_encode(svc, data, off, n, 0, enc, eoff));
                else if (is_svc)
                    CHK(qhuff_svc_decode(svc, huff, hoff, n, dec, doff, st));
                else if (!is_dec)
                    CHK(qhuff_encode_batch_host(plain, data, off, n, 0, enc,
                                                eoff));
                else
                    CHK(qhuff_decode_batch_host(plain, huff, hoff, n, dec,
                                                doff, st));
                if (i >= 0)
                    t[i] = now_us() - a;
            }
            static const char *nm[] = {"svc_encode_us", "svc_decode_us",
                                       "host_encode_us", "host_decode_us"};
            put(nm[p], stats(t, calls), 0);
            if (is_dec && (doff[n] != raw || memcmp(dec, data, raw)))
            {
                fprintf(stderr, "round trip mismatch (n=%u)\n", n);
                return 1;
            }
        }
        /* one literal per call, the reference's pattern */
        for (int p = 0; p < 2; ++p)
        {
            qhuff_ctx *cx = p ? plain : sc;
            unsigned char dst[256];
            for (int i = -50; i < calls; ++i)
            {
                dst[0] = 0;
                const double a = now_us();
                const int r = qhuff_enc_enc_str(cx, 7, dst, sizeof(dst),
                                                data + off[0], off[1] - off[0]);
                if (i >= 0)
                    t[i] = now_us() - a;
                if (r <= 0)
                {
                    fprintf(stderr, "enc_enc_str %d\n", r);
                    return 1;
                }
            }
            put(p ? "enc_str_plain_us" : "enc_str_svc_us", stats(t, calls), p);
        }
        printf("}");
        free(data), free(off), free(enc), free(dec), free(st), free(eoff);
        free(doff), free(huff), free(hoff);
    }
    {
        /* 20-string header blocks from T threads for 0.5 s each */
        uint8_t data[64 * 20 + 64];
        uint32_t off[21];
        qhuff_synth_batch(77, 20, 8, 64, (const uint8_t *) "abcdefghij-./", 13,
                          data, off);
        printf("}, \"threads_header_block_encode\": {");
        const int ts[] = {1, 2, 4, 8, 12, 16};
        for (unsigned j = 0; j < sizeof(ts) / sizeof(ts[0]); ++j)
        {
            pthread_t th[16];
            struct tp_arg ar[16];
            for (int i = 0; i < ts[j]; ++i)
            {
                ar[i] = (struct tp_arg){svc, data, off, 20, 0.5, 0};
                pthread_create(&th[i], NULL, tp_worker, &ar[i]);
            }
            long tot = 0;
            for (int i = 0; i < ts[j]; ++i)
            {
                pthread_join(th[i], NULL);
                tot += ar[i].calls;
            }
            printf("%s\"%d\": {\"blocks_per_s\": %.0f, \"strings_per_s\": %.0f}",
                   j ? ", " : "", ts[j], tot / 0.5, 20 * tot / 0.5);
        }
    }
    uint64_t served, launches, fb;
    qhuff_svc_stats(svc, &served, &launches, &fb);
    printf("}, \"svc_served\": %llu, \"svc_launches\": %llu, "
           "\"svc_fallbacks\": %llu}\n",
           (unsigned long long) served, (unsigned long long) launches,
           (unsigned long long) fb);
    qhuff_svc_close(svc);
    qhuff_close(sc);
    qhuff_close(plain);
    free(t);
    return 0;
}
