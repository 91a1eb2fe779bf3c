/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see qhuff_oracle.c header for the rule:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * it, as the checker; the product never does).
 *
 * CPU restatement of XXH32 as vendored by ls-qpack (deps/xxhash/xxhash.c,
 * xxHash r39-era API) and of the two header hashes lsqpack.c takes with it.
 * Pinned against the reference source itself: oracle/Makefile compiles
 * /root/reference/deps/xxhash/xxhash.c (one file, no generated code) into
 * oracle/_ref/libxxh32_ref.so, and tests/golden/make_xxh32_golden.py writes
 * its outputs to tests/golden/xxh32.json for the boxes without the reference.
 *
 *   oq_xxh32          xxhash.c:256-328  (XXH32_endian_align; primes 191-195)
 *   oq_xxh32_headers  lsqpack.c:1681-1685, 3268-3269, 3308-3309
 *                     (name hash seeded with LSQPACK_XXH_SEED, lsqpack.c:623;
 *                      name+value hash seeded with the name hash)
 */
#include <stdint.h>
#include <string.h>

#define P1 2654435761U
#define P2 2246822519U
#define P3 3266489917U
#define P4 668265263U
#define P5 374761393U

static inline uint32_t rotl (uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static inline uint32_t
le32 (const unsigned char *p)
{
    return (uint32_t) p[0] | (uint32_t) p[1] << 8 | (uint32_t) p[2] << 16
         | (uint32_t) p[3] << 24;
}

uint32_t
oq_xxh32 (const unsigned char *p, size_t len, uint32_t seed)
{
    const unsigned char *const end = p + len;
    uint32_t h;
    if (len >= 16)                                       /* xxhash.c:273-304 */
    {
        const unsigned char *const limit = end - 16;
        uint32_t v[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
        do
            for (int i = 0; i < 4; ++i, p += 4)
                v[i] = rotl(v[i] + le32(p) * P2, 13) * P1;
        while (p <= limit);
        h = rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
    }
    else
        h = seed + P5;                                   /* xxhash.c:305 */
    h += (uint32_t) len;                                 /* xxhash.c:307 */
    for (; p + 4 <= end; p += 4)                         /* xxhash.c:309-314 */
        h = rotl(h + le32(p) * P3, 17) * P4;
    for (; p < end; ++p)                                 /* xxhash.c:316-320 */
        h = rotl(h + *p * P5, 11) * P1;
    h ^= h >> 15;                                        /* xxhash.c:322-327 */
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

/* n headers, name i = buf[off[2i], off[2i+1]), value i = buf[off[2i+1],
 * off[2i+2]) */
void
oq_xxh32_headers (const unsigned char *buf, const uint32_t *off, uint32_t n,
                  uint32_t seed, uint32_t *name_hash, uint32_t *nameval_hash)
{
    for (uint32_t i = 0; i < n; ++i)
    {
        const uint32_t a = off[2 * i], m = off[2 * i + 1], b = off[2 * i + 2];
        name_hash[i] = oq_xxh32(buf + a, m - a, seed);
        nameval_hash[i] = oq_xxh32(buf + m, b - m, name_hash[i]);
    }
}
