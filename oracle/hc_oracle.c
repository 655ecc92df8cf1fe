/*
 * hc_oracle.c — CPU restatement of the dominiksalvet/huffman-codec codec path.
 *
 * TEST INFRASTRUCTURE ONLY (see hc_oracle.h). This is the checker the HIP path is compared
 * against; it is never part of the shipped library, the CLI or the measured path.
 *
 * Every function cites the reference file:line it restates (paths under /root/reference/src).
 * The restatement is pinned against the compiled reference (oracle/_ref/huffman-codec) by
 * tests/test_oracle.py and the fixtures in tests/golden/.
 */
#include "hc_oracle.h"

#include <stdlib.h>
#include <string.h>

void hco_free(void *p) { free(p); }

/* ------------------------------------------------------------------ diff model ---------- */

/* transform.cpp:220-229 — y[i] = x[i] - x[i-1] (mod 256), x[-1] = 0, over the linear stream */
void hco_diff_apply(uint8_t *v, uint64_t n)
{
    uint8_t last = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t x = v[i];
        v[i] = (uint8_t)(x - last);
        last = x;
    }
}

/* transform.cpp:231-239 — running sum mod 256 */
void hco_diff_revert(uint8_t *v, uint64_t n)
{
    uint8_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        acc = (uint8_t)(acc + v[i]);
        v[i] = acc;
    }
}

/* ------------------------------------------------------------------ MNP-5 RLE ----------- */

/* transform.cpp:241-279. Tag-less: after three equal literals one count byte (0..255 extra
 * copies) follows; a run is cut every 258 bytes; the final input byte is always a literal. */
uint64_t hco_rle_apply(const uint8_t *in, uint64_t n, uint8_t *out)
{
    uint64_t o = 0;
    uint8_t run_byte = 0;
    unsigned run = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t c = in[i];
        if (run != 0 && c == run_byte && i + 1 != n) { /* transform.cpp:252 */
            ++run;
            if (run <= 3) {
                out[o++] = c;
            } else if (run == 258) { /* transform.cpp:259-263 */
                out[o++] = 255;
                run = 0;
            }
        } else {
            if (run >= 3) out[o++] = (uint8_t)(run - 3); /* transform.cpp:267-270 */
            out[o++] = c;
            run_byte = c;
            run = 1;
        }
    }
    return o;
}

typedef struct {
    uint8_t byte; /* matchByte */
    int seen;     /* matchCount */
} rle_fsm;

/* transform.cpp:137-159 — one decoder step; returns the number of bytes it produces and
 * stores the ones that land below cap. */
static uint64_t rle_step(rle_fsm *st, uint8_t c, uint8_t *out, uint64_t pos, uint64_t cap)
{
    if (st->seen == 3) {
        for (unsigned r = 0; r < c; ++r)
            if (pos + r < cap) out[pos + r] = st->byte;
        st->seen = 0;
        return c;
    }
    if (pos < cap) out[pos] = c;
    if (c == st->byte) {
        st->seen++;
    } else {
        st->byte = c;
        st->seen = 1;
    }
    return 1;
}

/* transform.cpp:281-292 */
uint64_t hco_rle_revert(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap)
{
    rle_fsm st = {0, 0};
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) pos += rle_step(&st, in[i], out, pos, cap);
    return pos;
}

/* ------------------------------------------------------------------ adaptive block RLE -- */

static uint64_t ceil_div(uint64_t a, uint64_t b) { return a / b + (a % b != 0); }

/* transform.cpp:410-418 */
static uint64_t block_count(uint64_t w, uint64_t h, uint64_t b) { return ceil_div(w, b) * ceil_div(h, b); }

/* transform.cpp:25-62 — base offset and clipped extent of block i */
static void block_geom(uint64_t w, uint64_t h, uint64_t b, uint64_t i, uint64_t *base,
                       uint64_t *sx, uint64_t *sy)
{
    const uint64_t per_row = ceil_div(w, b);
    const uint64_t o = (i / per_row) * w * b + (i % per_row) * b;
    const uint64_t bx = o % w, by = o / w;
    *base = o;
    *sx = (bx + b > w) ? w - bx : b;
    *sy = (by + b > h) ? h - by : b;
}

/* transform.cpp:66-94 — horizontal = row-major inside the block, vertical = column-major */
static void block_gather(const uint8_t *m, uint64_t w, uint64_t base, uint64_t sx, uint64_t sy,
                         int horizontal, uint8_t *buf)
{
    uint64_t k = 0;
    if (horizontal) {
        for (uint64_t y = 0; y < sy; ++y)
            for (uint64_t x = 0; x < sx; ++x) buf[k++] = m[base + y * w + x];
    } else {
        for (uint64_t x = 0; x < sx; ++x)
            for (uint64_t y = 0; y < sy; ++y) buf[k++] = m[base + y * w + x];
    }
}

/* transform.cpp:191-216 (inverse of block_gather) */
static void block_scatter(uint8_t *m, uint64_t w, uint64_t base, uint64_t sx, uint64_t sy,
                          int horizontal, const uint8_t *buf)
{
    uint64_t k = 0;
    if (horizontal) {
        for (uint64_t y = 0; y < sy; ++y)
            for (uint64_t x = 0; x < sx; ++x) m[base + y * w + x] = buf[k++];
    } else {
        for (uint64_t x = 0; x < sx; ++x)
            for (uint64_t y = 0; y < sy; ++y) m[base + y * w + x] = buf[k++];
    }
}

static void put_be64(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (56 - 8 * i));
}

static uint64_t get_be64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}

uint64_t hco_adapt_bound(uint64_t n, uint64_t width)
{
    (void)width;
    /* header (24 + dir bytes of the B=8 tiling) + every block's RLE (<= 4/3 of it + 1) */
    return 24 + n / 64 + 64 + n + n / 3 + n / 64 + 64;
}

/* transform.cpp:97-134 + headers.cpp:18-63 for one block size; returns the stream length */
static uint64_t adapt_one(const uint8_t *m, uint64_t w, uint64_t h, uint64_t b, uint8_t *out,
                          uint8_t *scan, uint8_t *rle_h, uint8_t *rle_v)
{
    const uint64_t nb = block_count(w, h, b);
    const uint64_t hdr = 24 + ceil_div(nb, 8);
    put_be64(out, w);
    put_be64(out + 8, h);
    put_be64(out + 16, b);
    memset(out + 24, 0, hdr - 24);
    uint64_t o = hdr;
    for (uint64_t i = 0; i < nb; ++i) {
        uint64_t base, sx, sy;
        block_geom(w, h, b, i, &base, &sx, &sy);
        block_gather(m, w, base, sx, sy, 1, scan);
        const uint64_t lh = hco_rle_apply(scan, sx * sy, rle_h);
        block_gather(m, w, base, sx, sy, 0, scan);
        const uint64_t lv = hco_rle_apply(scan, sx * sy, rle_v);
        if (lh <= lv) { /* transform.cpp:113-117: tie -> horizontal (bit 1) */
            out[24 + i / 8] |= (uint8_t)(0x80u >> (i % 8));
            memcpy(out + o, rle_h, lh);
            o += lh;
        } else {
            memcpy(out + o, rle_v, lv);
            o += lv;
        }
    }
    return o;
}

/* transform.cpp:294-328 — try B = 8, 16, ... (<= 7 doublings, B <= W and B <= H); keep the
 * first strictly-smaller total (header + data) */
int hco_adapt_apply(const uint8_t *m, uint64_t width, uint64_t height, uint8_t *out,
                    uint64_t *out_len, uint64_t *best_block)
{
    if (width < 8 || height < 8) return 12; /* transform.cpp:300-304 */
    const uint64_t n = width * height;
    const uint64_t cap = hco_adapt_bound(n, width);
    uint8_t *cur = (uint8_t *)malloc(cap);
    uint8_t *scan = (uint8_t *)malloc(n + 16);
    uint8_t *rh = (uint8_t *)malloc(n + n / 3 + 16);
    uint8_t *rv = (uint8_t *)malloc(n + n / 3 + 16);
    uint64_t b = 8;
    uint64_t best = adapt_one(m, width, height, b, out, scan, rh, rv);
    *best_block = b;
    b *= 2;
    for (int step = 1; step <= 7 && b <= width && b <= height; ++step, b *= 2) {
        const uint64_t len = adapt_one(m, width, height, b, cur, scan, rh, rv);
        if (len < best) {
            memcpy(out, cur, len);
            best = len;
            *best_block = b;
        }
    }
    *out_len = best;
    free(cur);
    free(scan);
    free(rh);
    free(rv);
    return 0;
}

/* transform.cpp:330-361 + headers.cpp:65-105 + transform.cpp:162-187 */
int hco_adapt_revert(const uint8_t *in, uint64_t n, uint8_t **out, uint64_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    if (n < 24) return 10; /* headers.cpp:67-71 */
    const uint64_t w = get_be64(in), h = get_be64(in + 8), b = get_be64(in + 16);
    if (b == 0) return 100; /* reference: division by zero in getBlockCount */
    const uint64_t nb = block_count(w, h, b);
    const uint64_t dir_bytes = ceil_div(nb, 8);
    if (n - 24 < dir_bytes) return 11; /* headers.cpp:94-98 */
    if (w != 0 && h > (((uint64_t)1) << 36) / w) return 101; /* reference: bad_alloc */
    uint8_t *m = (uint8_t *)calloc(w * h + 1, 1);
    const uint64_t bw = b < w ? b : w, bh = b < h ? b : h;
    uint8_t *blk = (uint8_t *)malloc(bw * bh + 1);
    uint64_t pos = 24 + dir_bytes;
    for (uint64_t i = 0; i < nb; ++i) {
        uint64_t base, sx, sy;
        block_geom(w, h, b, i, &base, &sx, &sy);
        const uint64_t want = sx * sy;
        rle_fsm st = {0, 0};
        uint64_t got = 0;
        while (got < want) {
            if (pos >= n) { /* transform.cpp:170-174 */
                free(m);
                free(blk);
                return 14;
            }
            got += rle_step(&st, in[pos++], blk, got, want);
        }
        if (got != want) { /* transform.cpp:178-182 */
            free(m);
            free(blk);
            return 13;
        }
        const int horizontal = (in[24 + i / 8] >> (7 - i % 8)) & 1;
        block_scatter(m, w, base, sx, sy, horizontal, blk);
    }
    free(blk);
    if (pos != n) { /* transform.cpp:354-358 */
        free(m);
        return 15;
    }
    *out = m;
    *out_len = w * h;
    return 0;
}

/* ------------------------------------------------------------------ FGK, pointer form --- */

/* huffman.hpp:23-31: node number, weight, symbol, parent / left / right links */
typedef struct {
    uint16_t num;
    uint64_t weight;
    uint8_t symbol;
    int16_t up, lo, hi;
} fg_node;

typedef struct {
    fg_node n[513];
    int used;
    int root, nyt;
    int16_t leaf[256];
} fg_tree;

/* huffman.cpp:23-31 — a lone NYT root numbered 2*256 */
static void fg_init(fg_tree *t)
{
    t->used = 1;
    t->root = t->nyt = 0;
    t->n[0].num = 512;
    t->n[0].weight = 0;
    t->n[0].symbol = 0;
    t->n[0].up = t->n[0].lo = t->n[0].hi = -1;
    for (int i = 0; i < 256; ++i) t->leaf[i] = -1;
}

static int fg_leaf(const fg_tree *t, int x) { return t->n[x].lo < 0; } /* huffman.cpp:15-19 */

/* huffman.cpp:157-184 — pruned DFS: descend only through nodes heavier than f; among the
 * found nodes of weight f keep the highest number */
static int fg_leader(const fg_tree *t, int x, uint64_t f)
{
    const fg_node *d = &t->n[x];
    if (!fg_leaf(t, x) && d->weight > f) {
        const int a = fg_leader(t, d->lo, f);
        const int c = fg_leader(t, d->hi, f);
        if (a >= 0 && c >= 0) return t->n[a].num > t->n[c].num ? a : c;
        return a >= 0 ? a : c;
    }
    return d->weight == f ? x : -1;
}

/* huffman.cpp:186-217 — exchange two subtrees; the numbers stay with the positions */
static void fg_swap(fg_tree *t, int a, int c)
{
    const uint16_t num = t->n[a].num;
    t->n[a].num = t->n[c].num;
    t->n[c].num = num;
    const int pa = t->n[a].up, pc = t->n[c].up;
    const int a_left = t->n[pa].lo == a, c_left = t->n[pc].lo == c;
    if (a_left) t->n[pa].lo = (int16_t)c; else t->n[pa].hi = (int16_t)c;
    if (c_left) t->n[pc].lo = (int16_t)a; else t->n[pc].hi = (int16_t)a;
    t->n[a].up = (int16_t)pc;
    t->n[c].up = (int16_t)pa;
}

/* huffman.cpp:95-128 */
static void fg_update(fg_tree *t, uint8_t s)
{
    int x = t->leaf[s];
    if (x < 0) { /* split the NYT leaf: new NYT left (num-2), new symbol leaf right (num-1) */
        const int old = t->nyt;
        const int l = t->used++, r = t->used++;
        t->n[l].num = (uint16_t)(t->n[old].num - 2);
        t->n[r].num = (uint16_t)(t->n[old].num - 1);
        t->n[l].weight = t->n[r].weight = 0;
        t->n[l].symbol = 0;
        t->n[r].symbol = s;
        t->n[l].up = t->n[r].up = (int16_t)old;
        t->n[l].lo = t->n[l].hi = t->n[r].lo = t->n[r].hi = -1;
        t->n[old].lo = (int16_t)l;
        t->n[old].hi = (int16_t)r;
        t->nyt = l;
        t->leaf[s] = (int16_t)r;
        x = r;
    }
    while (x != t->root) {
        const int y = fg_leader(t, t->root, t->n[x].weight);
        if (y >= 0 && y != t->n[x].up && y != x) fg_swap(t, x, y);
        t->n[x].weight++;
        x = t->n[x].up;
    }
    t->n[x].weight++;
}

typedef struct {
    uint8_t *buf;
    uint64_t nbits;
} bit_sink;

static void sink_bit(bit_sink *w, unsigned bit)
{
    if (bit) w->buf[w->nbits >> 3] |= (uint8_t)(0x80u >> (w->nbits & 7));
    w->nbits++;
}

/* huffman.cpp:136-155 — emit the root-to-node path (collected leaf-up, then reversed) */
static void fg_path(const fg_tree *t, int x, bit_sink *w)
{
    unsigned char tmp[600];
    int d = 0;
    while (x != t->root) {
        const int p = t->n[x].up;
        tmp[d++] = (unsigned char)(t->n[p].lo != x);
        x = p;
    }
    while (d > 0) sink_bit(w, tmp[--d]);
}

uint64_t hco_fgk_bound(uint64_t n) { return n * 9 + 16; }

/* transform.cpp:363-384 with huffman.cpp:37-58 */
uint64_t hco_fgk_encode(const uint8_t *sym, uint64_t n, uint8_t *out)
{
    fg_tree *t = (fg_tree *)malloc(sizeof(fg_tree));
    fg_init(t);
    memset(out, 0, hco_fgk_bound(n));
    bit_sink w = {out, 0};
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t s = sym[i];
        if (t->leaf[s] < 0) {
            fg_path(t, t->nyt, &w);
            for (int k = 7; k >= 0; --k) sink_bit(&w, (s >> k) & 1);
        } else {
            fg_path(t, t->leaf[s], &w);
        }
        fg_update(t, s);
    }
    free(t);
    return w.nbits;
}

static unsigned bit_at(const uint8_t *b, uint64_t i) { return (b[i >> 3] >> (7 - (i & 7))) & 1; }

/* transform.cpp:386-406 with huffman.cpp:60-93 */
int hco_fgk_decode(const uint8_t *bits, uint64_t nbits, uint64_t count, uint8_t *sym)
{
    fg_tree *t = (fg_tree *)malloc(sizeof(fg_tree));
    fg_init(t);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < count; ++i) {
        int x = t->root;
        while (!fg_leaf(t, x)) {
            if (pos >= nbits) {
                free(t);
                return 9;
            }
            x = bit_at(bits, pos++) ? t->n[x].hi : t->n[x].lo;
        }
        uint8_t s = 0;
        if (x == t->nyt) {
            for (int k = 0; k < 8; ++k) {
                if (pos >= nbits) {
                    free(t);
                    return 9;
                }
                s = (uint8_t)((s << 1) | bit_at(bits, pos++));
            }
        } else {
            s = t->n[x].symbol;
        }
        fg_update(t, s);
        sym[i] = s;
    }
    free(t);
    return 0;
}

/* ------------------------------------------------------------------ FGK, slot form ------ */
/* SURVEY.md Appendix A.5. Position p in 0..512 carries the reference's node number p; the
 * root is always 512; siblings are the pairs (2k, 2k+1) with the left child even, so a code
 * bit is p & 1; weights are non-decreasing in p, so the pruned DFS of huffman.cpp:157-184
 * returns the highest p with the node's weight. */

enum { SL_INNER = 0x100, SL_NYT = 0x200 };

typedef struct {
    uint64_t weight[514]; /* [513] = sentinel above every weight */
    uint16_t up[513];     /* parent position of each position */
    uint16_t body[513];   /* symbol | SL_INNER + child pair | SL_NYT */
    uint16_t where[256];  /* symbol -> position; 0 = unseen (position 0 never holds a leaf) */
    int nyt;
} sl_tree;

static void sl_init(sl_tree *t)
{
    memset(t, 0, sizeof(*t));
    t->weight[513] = ~(uint64_t)0;
    t->body[512] = SL_NYT;
    t->nyt = 512;
}

static void sl_relink(sl_tree *t, uint16_t body, int pos)
{
    if (body & SL_INNER) {
        const int c = (body & 0xFF) * 2;
        t->up[c] = t->up[c + 1] = (uint16_t)pos;
    } else if (!(body & SL_NYT)) {
        t->where[body] = (uint16_t)pos;
    }
}

static void sl_split(sl_tree *t, uint8_t s)
{
    const int z = t->nyt;
    t->body[z] = (uint16_t)(SL_INNER | ((z - 2) >> 1));
    t->body[z - 2] = SL_NYT;
    t->body[z - 1] = s;
    t->weight[z - 2] = t->weight[z - 1] = 0;
    t->up[z - 2] = t->up[z - 1] = (uint16_t)z;
    t->where[s] = (uint16_t)(z - 1);
    t->nyt = z - 2;
}

static void sl_update(sl_tree *t, int x)
{
    while (x != 512) {
        const uint64_t f = t->weight[x];
        int lead = x;
        while (t->weight[lead + 1] == f) ++lead;
        if (lead != x && lead != t->up[x]) {
            const uint16_t a = t->body[x], c = t->body[lead];
            t->body[x] = c;
            t->body[lead] = a;
            sl_relink(t, c, x);
            sl_relink(t, a, lead);
            x = lead;
        }
        t->weight[x]++;
        x = t->up[x];
    }
    t->weight[512]++;
}

static void sl_path(const sl_tree *t, int x, bit_sink *w)
{
    unsigned char tmp[600];
    int d = 0;
    while (x != 512) {
        tmp[d++] = (unsigned char)(x & 1);
        x = t->up[x];
    }
    while (d > 0) sink_bit(w, tmp[--d]);
}

uint64_t hco_fgk_encode_slot(const uint8_t *sym, uint64_t n, uint8_t *out)
{
    sl_tree *t = (sl_tree *)malloc(sizeof(sl_tree));
    sl_init(t);
    memset(out, 0, hco_fgk_bound(n));
    bit_sink w = {out, 0};
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t s = sym[i];
        if (t->where[s] == 0) {
            sl_path(t, t->nyt, &w);
            for (int k = 7; k >= 0; --k) sink_bit(&w, (s >> k) & 1);
            sl_split(t, s);
        } else {
            sl_path(t, t->where[s], &w);
        }
        sl_update(t, t->where[s]);
    }
    free(t);
    return w.nbits;
}

int hco_fgk_decode_slot(const uint8_t *bits, uint64_t nbits, uint64_t count, uint8_t *sym)
{
    sl_tree *t = (sl_tree *)malloc(sizeof(sl_tree));
    sl_init(t);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < count; ++i) {
        int x = 512;
        while (t->body[x] & SL_INNER) {
            if (pos >= nbits) {
                free(t);
                return 9;
            }
            x = (t->body[x] & 0xFF) * 2 + (int)bit_at(bits, pos++);
        }
        uint8_t s;
        if (t->body[x] & SL_NYT) {
            s = 0;
            for (int k = 0; k < 8; ++k) {
                if (pos >= nbits) {
                    free(t);
                    return 9;
                }
                s = (uint8_t)((s << 1) | bit_at(bits, pos++));
            }
            sl_split(t, s);
        } else {
            s = (uint8_t)t->body[x];
        }
        sl_update(t, t->where[s]);
        sym[i] = s;
    }
    free(t);
    return 0;
}

/* ------------------------------------------------------------------ whole pipeline ------ */

/* main.cpp:39-87 (+ the width-0 check of main.cpp:195-199), headers.cpp:107-125 */
int hco_compress(const uint8_t *in, uint64_t n, int use_diff, int use_adapt, uint64_t width,
                 uint8_t **out, uint64_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    if (width == 0) return 4;
    if (use_adapt && n % width != 0) return 6;
    const uint64_t height = n / width;
    uint8_t *data = (uint8_t *)malloc(n + 1);
    if (n) memcpy(data, in, n);
    if (use_diff) hco_diff_apply(data, n);
    uint8_t *sym;
    uint64_t nsym;
    if (use_adapt) {
        uint64_t b;
        sym = (uint8_t *)malloc(hco_adapt_bound(n, width));
        const int st = hco_adapt_apply(data, width, height, sym, &nsym, &b);
        if (st) {
            free(sym);
            free(data);
            return st;
        }
    } else {
        sym = (uint8_t *)malloc(n + n / 3 + 8);
        nsym = hco_rle_apply(data, n, sym);
    }
    free(data);
    uint8_t *o = (uint8_t *)malloc(9 + hco_fgk_bound(nsym));
    const uint64_t nbits = hco_fgk_encode(sym, nsym, o + 9);
    free(sym);
    for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(nsym >> (8 * i)); /* little endian count */
    o[8] = (uint8_t)((use_diff ? 0x80 : 0) | (use_adapt ? 0x40 : 0));
    *out = o;
    *out_len = 9 + (nbits + 7) / 8;
    return 0;
}

/* main.cpp:90-128 */
int hco_decompress(const uint8_t *in, uint64_t n, uint8_t **out, uint64_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    if (n < 9) return 8; /* main.cpp:99-104 */
    uint64_t count = 0;
    for (int i = 7; i >= 0; --i) count = (count << 8) | in[i];
    const int use_diff = (in[8] >> 7) & 1, use_adapt = (in[8] >> 6) & 1;
    const uint64_t nbits = (n - 9) * 8;
    /* the first symbol costs >= 8 bits, each later one >= 1: more than this cannot decode,
     * and the reference stops with status 9 on such a stream */
    const uint64_t most = nbits >= 8 ? nbits - 7 : 0;
    if (count > most) return 9;
    uint8_t *sym = (uint8_t *)malloc(count + 1);
    int st = hco_fgk_decode(in + 9, nbits, count, sym);
    if (st) {
        free(sym);
        return st;
    }
    uint8_t *res;
    uint64_t len;
    if (use_adapt) {
        st = hco_adapt_revert(sym, count, &res, &len);
        free(sym);
        if (st) return st;
    } else {
        len = hco_rle_revert(sym, count, NULL, 0);
        res = (uint8_t *)malloc(len + 1);
        hco_rle_revert(sym, count, res, len);
        free(sym);
    }
    if (use_diff) hco_diff_revert(res, len);
    *out = res;
    *out_len = len;
    return 0;
}

/* ------------------------------------------------------------------ synthetic inputs ---- */

static uint64_t smix(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int64_t floor_div4(int64_t a) { return a >= 0 ? a / 4 : -((-a + 3) / 4); }

/* SURVEY.md Appendix D */
void hco_synth(int kind, uint64_t k, uint64_t width, uint64_t height, uint8_t *out)
{
    const uint64_t s = 24301ull * 1000003ull + k;
    const uint64_t T = 32;
    for (uint64_t y = 0; y < height; ++y) {
        for (uint64_t x = 0; x < width; ++x) {
            const uint64_t i = y * width + x;
            uint8_t v;
            if (kind == 0) {
                v = (uint8_t)(smix(s, i) & 0xFF);
            } else if (kind == 1) {
                v = (uint8_t)((x + 2 * y + k) & 0xFF);
            } else {
                const uint64_t t = (y / T) * (width / T) + x / T;
                const uint64_t th = smix(s ^ 0xABCDEF, t);
                const int64_t base = (int64_t)(th & 0xFF);
                const int64_t gx = (int64_t)((th >> 8) & 7) - 3;
                const int64_t gy = (int64_t)((th >> 11) & 7) - 3;
                const int64_t amp = (int64_t)((th >> 14) & 3);
                const int flat = ((th >> 16) & 3) == 0;
                const int64_t nz = (int64_t)((smix(s, i) & 7) % (uint64_t)(2 * amp + 1)) - amp;
                if (flat) {
                    v = (uint8_t)base;
                } else {
                    int64_t q = base + floor_div4((int64_t)(x % T) * gx + (int64_t)(y % T) * gy) + nz;
                    v = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
                }
            }
            out[i] = v;
        }
    }
}
