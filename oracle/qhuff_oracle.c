/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the ls-qpack v2.6.5 Huffman string-literal path
 * (/root/reference/lsqpack.c).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline.  The product (ls-qpack_amd/, libqhuff.so)
 * never links, loads or calls it.
 *
 * Why a restatement and not the reference itself: lsqpack.c includes
 * huff-tables.h (lsqpack.c:72), which is missing from the reference mount
 * (/root/reference/.MISSING_LARGE_BLOBS).  Building the reference would need a
 * stand-in for that file, so the reference is treated as unbuildable here.
 * This file re-derives the same four tables from the RFC 7541 Appendix B code
 * lengths and restates the reference's algorithms over them.  Parity of this
 * oracle is pinned by the reference's own known-answer tests and its committed
 * reference-encoded QPACK streams (tests/golden/).
 *
 * Functions and the reference lines they follow:
 *   oq_enc_str_size      lsqpack.c:5198-5210  (qenc_enc_str_size)
 *   oq_huffman_enc       lsqpack.c:5085-5195  (qenc_huffman_enc, pair table +
 *                                               per-byte tail + EOS padding)
 *   oq_enc_enc_str       lsqpack.c:839-876    (lsqpack_enc_enc_str) with
 *                        lsqpack.c:767-783    (lsqpack_val2len) and
 *                        lsqpack.c:819-836    (lsqpack_enc_int_nocheck)
 *   oq_huff_decode_full  lsqpack.c:3443-3517  (nibble FSM, resumable) with
 *                        lsqpack.c:5213-5231  (qdec_huff_dec4bits)
 *   oq_huff_decode       lsqpack.c:3520-3535  (dispatcher) ->
 *                        lsqpack.c:5234-5466  (huff_decode_fast)
 *   struct oq_retval     lsqpack.c:3420-3431  (struct huff_decode_retval)
 *   struct oq_dec_state  lsqpack.h:742-757    (lsqpack_huff_decode_state)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* RFC 7541 Appendix B code lengths, symbols 0..256. */
static const uint8_t rfc_len[257] = {
    13,23,28,28,28,28,28,28,28,24,30,28,28,30,28,28,28,28,28,28,28,28,30,28,28,28,28,28,28,28,28,28,
     6,10,10,12,13, 6, 8,11,10,10, 8,11, 8, 6, 6, 6, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8,15, 6,12,10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8,13,19,13,14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5, 6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7,15,11,14,13,28,
    20,22,20,20,22,22,22,23,22,23,23,23,23,23,24,23,24,24,22,23,24,23,23,23,23,21,22,23,22,23,23,24,
    22,21,20,22,22,23,23,21,23,22,22,24,21,22,23,23,21,21,22,21,23,22,23,23,20,22,22,22,23,22,22,23,
    26,26,20,19,22,23,22,25,26,26,26,27,27,26,24,25,19,21,26,27,27,26,27,24,21,21,26,26,28,27,27,27,
    20,24,20,21,22,21,21,23,22,22,25,25,24,24,26,23,26,27,26,26,27,27,27,27,27,28,27,27,27,27,27,26,
    30,
};

/* ---- table layouts (inferred from use sites) */

struct oq_code { uint32_t code; unsigned bits; };           /* encode_table */
struct oq_pair { unsigned lens; uint32_t code; };           /* hencs */
struct oq_nib  { uint8_t state, flags, sym; };              /* decode_tables */
struct oq_win  { uint8_t lens; uint8_t out[3]; };           /* hdecs */

enum { OQ_ACCEPTED = 1, OQ_SYM = 2, OQ_FAIL = 4 };           /* lsqpack.c:2579-2584 */
enum { OQ_OK, OQ_END_SRC, OQ_END_DST, OQ_ERROR };            /* lsqpack.c:3422-3428 */
#define OQ_SHORTEST_CODE 5                                   /* lsqpack.c:5072 */

struct oq_retval { int status; unsigned n_dst, n_src; };
struct oq_dec_state { int resume; uint8_t state, eos; };

static struct oq_code enc_tab[257];
static struct oq_pair *pair_tab;          /* 65536 entries */
static struct oq_nib nib_tab[256][16];
static struct oq_win *win_tab;            /* 65536 entries */

/* Binary code tree: node 0 is the root; child[n][b] >= 0 is an internal node,
 * child[n][b] = -1 - sym is a leaf.  256 internal nodes for 257 leaves. */
static int tree[256][2];
static int n_nodes;
static uint8_t node_accepts[256];

static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void
build_tables (void)
{
    int order[257], i, j;
    /* canonical code assignment: sort by (length, symbol) */
    for (i = 0; i < 257; ++i)
        order[i] = i;
    for (i = 1; i < 257; ++i)
        for (j = i; j > 0 && (rfc_len[order[j-1]] > rfc_len[order[j]]
                 || (rfc_len[order[j-1]] == rfc_len[order[j]]
                     && order[j-1] > order[j])); --j)
        {
            int t = order[j]; order[j] = order[j-1]; order[j-1] = t;
        }
    uint32_t code = 0;
    unsigned prev = rfc_len[order[0]];
    for (i = 0; i < 257; ++i)
    {
        unsigned s = order[i];
        code <<= rfc_len[s] - prev;
        prev = rfc_len[s];
        enc_tab[s].code = code;
        enc_tab[s].bits = rfc_len[s];
        ++code;
    }

    /* tree */
    memset(tree, 0, sizeof(tree));
    n_nodes = 1;
    for (int s = 0; s < 257; ++s)
    {
        int node = 0;
        for (int b = (int) enc_tab[s].bits - 1; b >= 0; --b)
        {
            int bit = (enc_tab[s].code >> b) & 1;
            if (b == 0)
                tree[node][bit] = -1 - s;
            else
            {
                if (tree[node][bit] == 0)
                {
                    tree[n_nodes][0] = tree[n_nodes][1] = 0;
                    tree[node][bit] = n_nodes++;
                }
                node = tree[node][bit];
            }
        }
    }
    /* accepting states: root, or an all-ones path of depth <= 7 (RFC 7541
     * 5.2: padding is a prefix of EOS no longer than 7 bits) */
    memset(node_accepts, 0, sizeof(node_accepts));
    {
        int node = 0;
        node_accepts[0] = 1;
        for (int d = 1; d <= 7; ++d)
        {
            node = tree[node][1];
            node_accepts[node] = 1;
        }
    }

    /* nibble FSM, lsqpack.c:5213-5231 consumes it */
    for (int st = 0; st < n_nodes; ++st)
        for (int nib = 0; nib < 16; ++nib)
        {
            int node = st, flags = 0, sym = 0;
            for (int b = 3; b >= 0; --b)
            {
                int nx = tree[node][(nib >> b) & 1];
                if (nx < 0)
                {
                    int s = -1 - nx;
                    if (s == 256) { flags = OQ_FAIL; node = 0; break; }
                    flags |= OQ_SYM;
                    sym = s;
                    node = 0;
                }
                else
                    node = nx;
            }
            if (!(flags & OQ_FAIL) && node_accepts[node])
                flags |= OQ_ACCEPTED;
            nib_tab[st][nib].state = (uint8_t) node;
            nib_tab[st][nib].flags = (uint8_t) flags;
            nib_tab[st][nib].sym = (uint8_t) sym;
        }

    /* pair encoder, lsqpack.c:5103-5139.  Index = 2-byte little-endian load
     * of the pair (first byte in the low half).  Pairs longer than 32 bits do
     * not fit the 32-bit code field and are marked lens = 64 (fall back). */
    pair_tab = malloc(sizeof(*pair_tab) * 65536);
    for (unsigned idx = 0; idx < 65536; ++idx)
    {
        const struct oq_code *a = &enc_tab[idx & 0xff], *b = &enc_tab[idx >> 8];
        unsigned l = a->bits + b->bits;
        if (l <= 32)
        {
            pair_tab[idx].lens = l;
            pair_tab[idx].code = (uint32_t)
                            (((uint64_t) a->code << b->bits) | b->code);
        }
        else
        {
            pair_tab[idx].lens = 64;
            pair_tab[idx].code = 0;
        }
    }

    /* 16-bit window decoder, lsqpack.c:5311-5358: greedily decode every
     * complete symbol in the window (at most 3, shortest code is 5 bits).
     * lens = bits_consumed << 2 | n_out; 0 means the first code is longer
     * than 16 bits (slow path). */
    win_tab = malloc(sizeof(*win_tab) * 65536);
    for (unsigned w = 0; w < 65536; ++w)
    {
        unsigned used = 0, n = 0, consumed = 0;
        int node = 0;
        struct oq_win e = { 0, { 0, 0, 0 } };
        while (used < 16 && n < 3)
        {
            int nx = tree[node][(w >> (15 - used)) & 1];
            ++used;
            if (nx < 0)
            {
                int s = -1 - nx;
                if (s == 256)
                    break;
                e.out[n++] = (uint8_t) s;
                consumed = used;
                node = 0;
            }
            else
                node = nx;
        }
        e.lens = (uint8_t) (n ? (consumed << 2) | n : 0);
        win_tab[w] = e;
    }
}

void
oq_init (void)
{
    pthread_once(&init_once, build_tables);
}

__attribute__((constructor)) static void
oq_ctor (void)
{
    oq_init();
}

/* ---- encoder ---------------------------------------------------------- */

unsigned
oq_enc_str_size (const unsigned char *str, unsigned len)
{
    unsigned bits = 0;
    for (unsigned i = 0; i < len; ++i)
        bits += enc_tab[str[i]].bits;
    return (bits + 7) / 8;
}

static inline unsigned char *
put64 (unsigned char *dst, uint64_t v)
{
    for (int sh = 56; sh >= 0; sh -= 8)
        *dst++ = (unsigned char) (v >> sh);
    return dst;
}

unsigned char *
oq_huffman_enc (const unsigned char *src, const unsigned char *const end,
                unsigned char *dst)
{
    uint64_t acc = 0;
    unsigned used = 0;

    /* pair-table body: runs while a full 64-bit accumulator of the shortest
     * codes plus one pair cannot run past the end (lsqpack.c:5103) */
    while (src + 64 / OQ_SHORTEST_CODE + 2 < end)
    {
        uint16_t idx;
        const struct oq_pair *p;
        memcpy(&idx, src, 2);
        p = &pair_tab[idx];
        src += 2;
        while (used + p->lens < 64)
        {
            acc = (acc << p->lens) | p->code;
            used += p->lens;
            memcpy(&idx, src, 2);
            p = &pair_tab[idx];
            src += 2;
        }
        if (p->lens >= 64)
        {
            src -= 2;
            break;
        }
        acc <<= 64 - used;
        used = p->lens - (64 - used);
        acc |= (uint64_t) p->code >> used;
        dst = put64(dst, acc);
        acc = p->code;
    }

    /* per-byte tail (lsqpack.c:5142-5169) */
    while (src != end)
    {
        const struct oq_code c = enc_tab[*src++];
        if (used + c.bits < 64)
        {
            acc = (acc << c.bits) | c.code;
            used += c.bits;
        }
        else
        {
            acc <<= 64 - used;
            used = c.bits - (64 - used);
            acc |= (uint64_t) c.code >> used;
            dst = put64(dst, acc);
            acc = c.code;
        }
    }

    /* pad the last partial byte with the EOS prefix (all ones),
     * lsqpack.c:5171-5189 */
    if (used)
    {
        unsigned total = (used + 7) & ~7u, pad = total - used;
        acc = (acc << pad) | ((1u << pad) - 1);
        for (int sh = (int) total - 8; sh >= 0; sh -= 8)
            *dst++ = (unsigned char) (acc >> sh);
    }
    return dst;
}

static unsigned
val2len (uint64_t v, unsigned prefix_bits)                 /* lsqpack.c:767 */
{
    uint64_t mask = (1ULL << prefix_bits) - 1;
    unsigned n = 1;
    if (v < mask)
        return 1;
    v -= mask;
    do
    {
        ++n;
        v >>= 7;
    }
    while (v);
    return n;
}

static void
put_int (unsigned char *dst, uint64_t v, unsigned prefix_bits) /* 819-836 */
{
    uint64_t mask = (1ULL << prefix_bits) - 1;
    if (v < mask)
    {
        *dst |= (unsigned char) v;
        return;
    }
    *dst++ |= (unsigned char) mask;
    v -= mask;
    while (v >= 128)
    {
        *dst++ = (unsigned char) (0x80 | (v & 0x7f));
        v >>= 7;
    }
    *dst = (unsigned char) v;
}

int
oq_enc_enc_str (unsigned prefix_bits, unsigned char *dst, size_t dst_len,
                const unsigned char *str, unsigned len)
{
    unsigned hlen = oq_enc_str_size(str, len);
    int huff = hlen < len;                       /* strict <, lsqpack.c:848 */
    unsigned plen = huff ? hlen : len;
    unsigned lsz = val2len(plen, prefix_bits);
    if ((size_t) lsz + plen > dst_len)
        return -1;
    dst[0] &= (unsigned char) ~((1u << (prefix_bits + 1)) - 1);
    if (huff)
        dst[0] |= (unsigned char) (1u << prefix_bits);
    put_int(dst, plen, prefix_bits);
    if (huff)
        oq_huffman_enc(str, str + len, dst + lsz);
    else
        memcpy(dst + lsz, str, len);
    return (int) (lsz + plen);
}

/* ---- decoder ---------------------------------------------------------- */

static inline int
nib_step (unsigned nib, unsigned char **dst, struct oq_dec_state *st)
{
    const struct oq_nib e = nib_tab[st->state][nib];
    if (e.flags & OQ_FAIL)
        return -1;
    if (e.flags & OQ_SYM)
        *(*dst)++ = e.sym;
    st->state = e.state;
    st->eos = (e.flags & OQ_ACCEPTED) != 0;
    return 0;
}

struct oq_retval
oq_huff_decode_full (const unsigned char *src, int src_len,
                     unsigned char *dst, int dst_len,
                     struct oq_dec_state *st, int final)
{
    const unsigned char *p = src, *const pend = src + src_len;
    unsigned char *d = dst, *const dend = dst + dst_len;
    struct oq_retval rv = { OQ_ERROR, 0, 0 };

    if (dst_len == 0)
    {
        rv.status = OQ_END_DST;
        return rv;
    }
    /* resume points: 0 fresh, 1 between bytes, 2 before the high nibble,
     * 3 before the low nibble (lsqpack.c:3460-3499) */
    if (st->resume == 0)
    {
        st->state = 0;
        st->eos = 1;
        st->resume = 1;
    }
    int at = st->resume;
    while (p != pend)
    {
        if (at <= 2)
        {
            if (at == 1 && d == dend)
            {
                st->resume = 2;
                rv.status = OQ_END_DST;
                rv.n_dst = (unsigned) dst_len;
                rv.n_src = (unsigned) (p - src);
                return rv;
            }
            if (nib_step(*p >> 4, &d, st))
                return (struct oq_retval) { OQ_ERROR, 0, 0 };
            if (d == dend)
            {
                st->resume = 3;
                rv.status = OQ_END_DST;
                rv.n_dst = (unsigned) dst_len;
                rv.n_src = (unsigned) (p - src);
                return rv;
            }
        }
        if (nib_step(*p & 0xf, &d, st))
            return (struct oq_retval) { OQ_ERROR, 0, 0 };
        ++p;
        at = 1;
    }
    rv.n_dst = (unsigned) (d - dst);
    rv.n_src = (unsigned) (p - src);
    if (final)
        rv.status = st->eos ? OQ_OK : OQ_ERROR;
    else
    {
        st->resume = 1;
        rv.status = OQ_END_SRC;
    }
    return rv;
}

static inline void
emit_win (unsigned char **d, const struct oq_win *w)
{
    unsigned n = w->lens & 3;
    for (unsigned i = 0; i < n; ++i)
        *(*d)++ = w->out[i];
}

/* lsqpack.c:5234-5466.  Complete-string fast path over the 16-bit window
 * table; a code longer than 16 bits sends the remainder to the nibble FSM
 * after backing up to the last byte-aligned symbol boundary. */
static struct oq_retval
huff_decode_fast (const unsigned char *src, int src_len,
                  unsigned char *dst, int dst_len,
                  struct oq_dec_state *st, int final)
{
    const unsigned char *p = src, *const pend = src + src_len;
    unsigned char *d = dst, *const dend = dst + dst_len;
    uint64_t buf = 0;
    unsigned avail = 0;
    struct oq_win w;
    const struct oq_retval err = { OQ_ERROR, 0, 0 };

    for (;;)
    {
        /* refill the 64-bit buffer with whole bytes */
        if (p < pend)
            while (p < pend && avail <= 56)
            {
                buf = (buf << 8) | *p++;
                avail += 8;
            }
        else
            break;

        if (dend - d >= 64 / OQ_SHORTEST_CODE && avail >= 16)
        {
            do
            {
                w = win_tab[(uint16_t) (buf >> (avail - 16))];
                d[0] = w.out[0];
                d[1] = w.out[1];
                d[2] = w.out[2];
                d += w.lens & 3;
                avail -= w.lens >> 2;
            }
            while (avail >= 16 && w.lens);
            if (avail < 16)
                continue;
            goto slow_path;
        }
        while (avail >= 16)
        {
            w = win_tab[(uint16_t) (buf >> (avail - 16))];
            unsigned n = w.lens & 3;
            if (n && d + n <= dend)
            {
                emit_win(&d, &w);
                avail -= w.lens >> 2;
            }
            else if (d + n > dend)
                goto dst_ended;
            else
                goto slow_path;
        }
    }

    /* tail: fewer than 16 bits left; pad the window with ones (EOS) */
    if (avail >= OQ_SHORTEST_CODE)
    {
        uint16_t idx = (uint16_t) (buf << (16 - avail));
        idx |= (uint16_t) ((1u << (16 - avail)) - 1);
        if (idx == 0xFFFF && avail < 8)
            goto done;              /* nothing but EOS padding is left */
        w = win_tab[idx];
        unsigned n = w.lens & 3;
        if ((unsigned) (w.lens >> 2) > avail)
            return err;             /* a symbol would eat padding bits */
        if (n && d + n <= dend)
        {
            emit_win(&d, &w);
            avail -= w.lens >> 2;
        }
        else if (d + n > dend)
            goto dst_ended;
        else
            return err;
    }
    if (avail >= 8)                 /* padding longer than 7 bits */
        return err;
    if (avail > 0 && (buf & ((1u << avail) - 1)) != ((1u << avail) - 1))
        return err;                 /* padding is not the EOS prefix */
  done:
    return (struct oq_retval) { OQ_OK, (unsigned) (d - dst),
                                (unsigned) (p - src) };

  dst_ended:
    while ((avail & 7) && d > dst)
        avail += enc_tab[*--d].bits;
    p -= avail >> 3;
    return (struct oq_retval) { OQ_END_DST, (unsigned) (d - dst),
                                (unsigned) (p - src) };

  slow_path:
    while ((avail & 7) && d > dst)
        avail += enc_tab[*--d].bits;
    p -= avail >> 3;
    {
        struct oq_retval rv = oq_huff_decode_full(p, (int) (pend - p), d,
                                              (int) (dend - d), st, final);
        if (rv.status == OQ_OK || rv.status == OQ_END_DST)
        {
            rv.n_dst += (unsigned) (d - dst);
            rv.n_src += (unsigned) (p - src);
        }
        return rv;
    }
}

struct oq_retval
oq_huff_decode (const unsigned char *src, int src_len, unsigned char *dst,
                int dst_len, struct oq_dec_state *st, int final)
{
    if (st->resume == 0 && final)
        return huff_decode_fast(src, src_len, dst, dst_len, st, final);
    return oq_huff_decode_full(src, src_len, dst, dst_len, st, final);
}

/* ---- batch drivers (tests + cpu_baseline) ------------------------------
 *
 * Batch layout shared with the product C-ABI (include/qhuff.h): strings are
 * packed back to back; in_off has n+1 entries (exclusive offsets).  Output
 * offsets are the exclusive scan of per-string output sizes, written to
 * out_off[0..n].
 *
 * mode: 0 = Huffman payload only (qenc_huffman_enc output, forced);
 *       3/5/7 = lsqpack_enc_enc_str(prefix_bits = mode) literal, first byte's
 *       bits above the prefix cleared (dst[0] = 0 before the call).
 */

unsigned long long
oq_encode_sizes (const unsigned char *in, const uint32_t *in_off, uint32_t n,
                 unsigned mode, uint32_t *out_off)
{
    unsigned long long tot = 0;
    for (uint32_t i = 0; i < n; ++i)
    {
        const unsigned char *s = in + in_off[i];
        unsigned len = in_off[i + 1] - in_off[i];
        unsigned h = oq_enc_str_size(s, len);
        unsigned sz;
        if (mode == 0)
            sz = h;
        else
        {
            unsigned plen = h < len ? h : len;
            sz = val2len(plen, mode) + plen;
        }
        out_off[i] = (uint32_t) tot;
        tot += sz;
    }
    out_off[n] = (uint32_t) tot;
    return tot;
}

void
oq_encode_batch (const unsigned char *in, const uint32_t *in_off, uint32_t n,
                 unsigned mode, unsigned char *out, const uint32_t *out_off)
{
    for (uint32_t i = 0; i < n; ++i)
    {
        const unsigned char *s = in + in_off[i];
        unsigned len = in_off[i + 1] - in_off[i];
        unsigned char *d = out + out_off[i];
        if (mode == 0)
            oq_huffman_enc(s, s + len, d);
        else
        {
            d[0] = 0;
            oq_enc_enc_str(mode, d, out_off[i + 1] - out_off[i], s, len);
        }
    }
}

/* Decode each string with the complete-string dispatcher (resume 0, final 1).
 * out must hold out_cap bytes per string slot at out_slot_off[i]; decoded
 * bytes are compacted into out (exclusive scan) and out_off[0..n] written.
 * status[i] = 0 OK, 1 ERROR (error strings contribute 0 bytes). */
int
oq_decode_batch (const unsigned char *in, const uint32_t *in_off, uint32_t n,
                 unsigned char *out, uint32_t *out_off, uint8_t *status,
                 int use_full)
{
    uint64_t tot = 0;
    int n_err = 0;
    for (uint32_t i = 0; i < n; ++i)
    {
        unsigned len = in_off[i + 1] - in_off[i];
        unsigned cap = len * 8 / 5 + 1;
        struct oq_dec_state st = { 0, 0, 0 };
        struct oq_retval rv = use_full
            ? oq_huff_decode_full(in + in_off[i], (int) len, out + tot,
                                  (int) cap, &st, 1)
            : oq_huff_decode(in + in_off[i], (int) len, out + tot, (int) cap,
                             &st, 1);
        out_off[i] = (uint32_t) tot;
        if (rv.status == OQ_OK)
        {
            status[i] = 0;
            tot += rv.n_dst;
        }
        else
        {
            status[i] = 1;
            ++n_err;
        }
    }
    out_off[n] = (uint32_t) tot;
    return n_err;
}

/* ---- threaded CPU baseline ---------------------------------------------
 * Mirrors SURVEY.md section 8(d): per-string lsqpack_enc_enc_str(7, slot,
 * 128, ...) and lsqpack_huff_decode(payload, len, slot, 128, state0, 1) into
 * private fixed-stride slots, static contiguous shards per thread. */

struct bench_arg
{
    const unsigned char *in;
    const uint32_t *in_off;
    uint32_t lo, hi;
    unsigned slot;
    int op;                  /* 0 enc_enc_str(7), 1 huff_decode, 2 _full */
    unsigned long long sink;
};

static void *
bench_worker (void *vp)
{
    struct bench_arg *a = vp;
    unsigned char *slot = malloc(a->slot);
    unsigned long long sink = 0;
    for (uint32_t i = a->lo; i < a->hi; ++i)
    {
        const unsigned char *s = a->in + a->in_off[i];
        unsigned len = a->in_off[i + 1] - a->in_off[i];
        if (a->op == 0)
        {
            slot[0] = 0;
            sink += (unsigned) oq_enc_enc_str(7, slot, a->slot, s, len);
        }
        else
        {
            struct oq_dec_state st = { 0, 0, 0 };
            struct oq_retval rv = a->op == 1
                ? oq_huff_decode(s, (int) len, slot, (int) a->slot, &st, 1)
                : oq_huff_decode_full(s, (int) len, slot, (int) a->slot,
                                      &st, 1);
            sink += rv.n_dst + (unsigned) rv.status;
        }
    }
    a->sink = sink + slot[0];
    free(slot);
    return NULL;
}

/* Returns wall seconds for one pass over strings [0, n) with nthreads. */
double
oq_bench_pass (const unsigned char *in, const uint32_t *in_off, uint32_t n,
               int op, int nthreads, unsigned slot_bytes,
               unsigned long long *sink_out)
{
    pthread_t th[256];
    struct bench_arg args[256];
    struct timespec t0, t1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; ++t)
    {
        args[t].in = in;
        args[t].in_off = in_off;
        args[t].lo = (uint32_t) ((uint64_t) n * t / nthreads);
        args[t].hi = (uint32_t) ((uint64_t) n * (t + 1) / nthreads);
        args[t].slot = slot_bytes;
        args[t].op = op;
        args[t].sink = 0;
        if (nthreads > 1)
            pthread_create(&th[t], NULL, bench_worker, &args[t]);
    }
    if (nthreads == 1)
        bench_worker(&args[0]);
    unsigned long long sink = 0;
    for (int t = 0; t < nthreads; ++t)
    {
        if (nthreads > 1)
            pthread_join(th[t], NULL);
        sink += args[t].sink;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (sink_out)
        *sink_out = sink;
    return (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* table accessors for tests */
void
oq_code_of (unsigned sym, uint32_t *code, unsigned *bits)
{
    *code = enc_tab[sym].code;
    *bits = enc_tab[sym].bits;
}
