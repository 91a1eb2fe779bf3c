/*
 * qhuff_hook.c -- see qhuff_hook.h.  Two open-addressing tables keyed by
 * string pointer; each batch call codes all entries in one GPU launch
 * (qhuff_encode_batch_host / qhuff_decode_literals_host).
 */
#include "qhuff_hook.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

struct slot
{
    const unsigned char *key;       /* string / payload pointer, NULL = free */
    unsigned len;
    unsigned idx;
};

struct table
{
    struct slot *s;
    unsigned mask;
};

struct qhuff_memo
{
    qhuff_ctx *ctx;
    /* encoder: the strings (copied, to check they did not change), their
     * payloads */
    struct table et;
    uint8_t *e_str, *e_huf;
    uint32_t *e_str_off, *e_huf_off;
    /* decoder: the Huffman payloads (copied, to check they did not change:
     * a receive buffer reused at the same address must not hit), decoded
     * strings and status per literal */
    struct table dt;
    uint8_t *d_src, *d_out, *d_st;
    uint32_t *d_src_off, *d_off;
};

static __thread struct qhuff_memo *t_memo;

static unsigned
hash_ptr(const unsigned char *p, unsigned len)
{
    uint64_t h = (uint64_t) (uintptr_t) p * 0x9e3779b97f4a7c15ull ^ len;
    return (unsigned) (h >> 32);
}

static int
table_init(struct table *t, unsigned n)
{
    unsigned cap = 16;
    while (cap < 2 * n)
        cap <<= 1;
    free(t->s);
    t->s = calloc(cap, sizeof *t->s);
    t->mask = cap - 1;
    return t->s ? 0 : -1;
}

static void
table_put(struct table *t, const unsigned char *key, unsigned len,
          unsigned idx)
{
    unsigned i = hash_ptr(key, len) & t->mask;
    while (t->s[i].key && !(t->s[i].key == key && t->s[i].len == len))
        i = (i + 1) & t->mask;
    t->s[i].key = key;          /* a repeated key keeps its last entry */
    t->s[i].len = len;
    t->s[i].idx = idx;
}

static const struct slot *
table_get(const struct table *t, const unsigned char *key, unsigned len)
{
    if (!t->s)
        return NULL;
    unsigned i = hash_ptr(key, len) & t->mask;
    while (t->s[i].key)
    {
        if (t->s[i].key == key && t->s[i].len == len)
            return &t->s[i];
        i = (i + 1) & t->mask;
    }
    return NULL;
}

struct qhuff_memo *
qhuff_memo_new(qhuff_ctx *ctx)
{
    struct qhuff_memo *m = calloc(1, sizeof *m);
    if (m)
        m->ctx = ctx;
    return m;
}

static void
enc_clear(struct qhuff_memo *m)
{
    free(m->e_str);
    free(m->e_huf);
    free(m->e_str_off);
    free(m->e_huf_off);
    free(m->et.s);
    m->e_str = m->e_huf = NULL;
    m->e_str_off = m->e_huf_off = NULL;
    m->et.s = NULL;
}

static void
dec_clear(struct qhuff_memo *m)
{
    free(m->d_src);
    free(m->d_src_off);
    free(m->d_out);
    free(m->d_st);
    free(m->d_off);
    free(m->dt.s);
    m->d_src = m->d_out = m->d_st = NULL;
    m->d_src_off = m->d_off = NULL;
    m->dt.s = NULL;
}

void
qhuff_memo_free(struct qhuff_memo *m)
{
    if (!m)
        return;
    if (t_memo == m)
        t_memo = NULL;
    enc_clear(m);
    dec_clear(m);
    free(m);
}

int
qhuff_memo_encode(struct qhuff_memo *m, const unsigned char *const *strs,
                  const unsigned *lens, unsigned n)
{
    enc_clear(m);
    uint64_t total = 0;
    for (unsigned i = 0; i < n; ++i)
        total += lens[i];
    if (total >= 0xffffffffull)
        return QHUFF_ERANGE;
    const uint64_t hb = qhuff_encode_bound(total, n, QHUFF_ENC_PAYLOAD);
    m->e_str = malloc(total ? total : 1);
    m->e_huf = malloc(hb ? hb : 1);
    m->e_str_off = malloc((n + 1) * sizeof *m->e_str_off);
    m->e_huf_off = malloc((n + 1) * sizeof *m->e_huf_off);
    if (!m->e_str || !m->e_huf || !m->e_str_off || !m->e_huf_off
            || table_init(&m->et, n))
    {
        enc_clear(m);
        return QHUFF_ENOMEM;
    }
    uint32_t o = 0;
    for (unsigned i = 0; i < n; ++i)
    {
        m->e_str_off[i] = o;
        memcpy(m->e_str + o, strs[i], lens[i]);
        o += lens[i];
    }
    m->e_str_off[n] = o;
    int rc = qhuff_encode_batch_host(m->ctx, m->e_str, m->e_str_off, n,
                                     QHUFF_ENC_PAYLOAD, m->e_huf,
                                     m->e_huf_off);
    if (rc != QHUFF_OK)
    {
        enc_clear(m);
        return rc;
    }
    for (unsigned i = 0; i < n; ++i)
        table_put(&m->et, strs[i], lens[i], i);
    return QHUFF_OK;
}

int
qhuff_memo_decode(struct qhuff_memo *m, const unsigned char *buf,
                  const struct qhuff_literal *lits, unsigned n)
{
    dec_clear(m);
    const uint64_t ob = qhuff_literals_bound(lits, n);
    uint64_t sb = 0;
    for (unsigned i = 0; i < n; ++i)
        sb += lits[i].huffman ? lits[i].len : 0;
    if (sb >= 0xffffffffull)
        return QHUFF_ERANGE;
    m->d_src = malloc(sb ? sb : 1);
    m->d_src_off = malloc((n + 1) * sizeof *m->d_src_off);
    m->d_out = malloc(ob ? ob : 1);
    m->d_st = malloc(n ? n : 1);
    m->d_off = malloc((n + 1) * sizeof *m->d_off);
    if (!m->d_src || !m->d_src_off || !m->d_out || !m->d_st || !m->d_off
            || table_init(&m->dt, n))
    {
        dec_clear(m);
        return QHUFF_ENOMEM;
    }
    int rc = qhuff_decode_literals_host(m->ctx, buf, lits, n, m->d_out,
                                        m->d_off, m->d_st);
    if (rc != QHUFF_OK)
    {
        dec_clear(m);
        return rc;
    }
    uint32_t o = 0;
    for (unsigned i = 0; i < n; ++i)
    {
        m->d_src_off[i] = o;
        if (lits[i].huffman)        /* the reference decodes only these */
        {
            memcpy(m->d_src + o, buf + lits[i].pos, lits[i].len);
            o += lits[i].len;
            table_put(&m->dt, buf + lits[i].pos, lits[i].len, i);
        }
    }
    m->d_src_off[n] = o;
    return QHUFF_OK;
}

void
lsqpack_qhuff_use(struct qhuff_memo *m)
{
    t_memo = m;
}

/* the memo entry of str if its bytes are the ones that were coded */
static int
enc_find(const unsigned char *str, unsigned len)
{
    const struct qhuff_memo *m = t_memo;
    const struct slot *s = m ? table_get(&m->et, str, len) : NULL;
    if (!s || memcmp(m->e_str + m->e_str_off[s->idx], str, len) != 0)
        return -1;
    return (int) s->idx;
}

int
lsqpack_qhuff_payload(const unsigned char *str, unsigned str_len,
                      const unsigned char **huff, unsigned *huff_len)
{
    const int i = enc_find(str, str_len);
    if (i < 0)
        return 0;
    *huff = t_memo->e_huf + t_memo->e_huf_off[i];
    *huff_len = t_memo->e_huf_off[i + 1] - t_memo->e_huf_off[i];
    return 1;
}

int
lsqpack_qhuff_enc_lookup(unsigned prefix_bits, unsigned char *dst,
                         size_t dst_len, const unsigned char *str,
                         unsigned str_len)
{
    const unsigned char *huff;
    unsigned huff_len;
    if (!lsqpack_qhuff_payload(str, str_len, &huff, &huff_len))
        return LSQPACK_QHUFF_MISS;
    return qhuff_frame_literal(prefix_bits, dst, dst_len, str, str_len, huff,
                               huff_len);
}

int
lsqpack_qhuff_enc_str_size(const unsigned char *str, unsigned str_len)
{
    const unsigned char *huff;
    unsigned huff_len;
    if (!lsqpack_qhuff_payload(str, str_len, &huff, &huff_len))
        return -1;
    return (int) huff_len;
}

int
lsqpack_qhuff_dec_lookup(const unsigned char *src, int src_len,
                         unsigned char *dst, int dst_len,
                         struct qhuff_decode_retval *rv)
{
    const struct qhuff_memo *m = t_memo;
    if (!m || src_len < 0 || dst_len < 0)
        return 0;
    const struct slot *s = table_get(&m->dt, src, (unsigned) src_len);
    if (!s || m->d_st[s->idx] != QHUFF_DEC_OK
            || memcmp(m->d_src + m->d_src_off[s->idx], src, (size_t) src_len))
        return 0;                   /* not memoised, or the bytes changed */
    const uint32_t n = m->d_off[s->idx + 1] - m->d_off[s->idx];
    /* With room to spare the reference returns OK whichever of its decoders
     * runs (neither can reach its dst_ended condition); at n >= dst_len its
     * END_DST rules decide, so the reference code answers. */
    if (n >= (uint32_t) dst_len)
        return 0;
    memcpy(dst, m->d_out + m->d_off[s->idx], n);
    rv->status = QHUFF_HUFF_DEC_OK;
    rv->n_dst = n;
    rv->n_src = (unsigned) src_len;
    return 1;
}
