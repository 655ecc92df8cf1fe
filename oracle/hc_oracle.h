/*
 * hc_oracle.h — CPU restatement of dominiksalvet/huffman-codec (reference @ /root/reference).
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (huffman-codec_amd/, include/) links,
 * loads or calls this. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, and only as the checker. Parity of this restatement is pinned against the real
 * reference binary (oracle/_ref/huffman-codec, built from /root/reference/src by
 * oracle/Makefile) through tests/golden/ (see tests/test_oracle.py).
 *
 * Status codes are the reference's process exit codes; 0 = success.
 */
#ifndef HC_ORACLE_H
#define HC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* transform.cpp:220-229 / 231-239 (in place) */
void hco_diff_apply(uint8_t *v, uint64_t n);
void hco_diff_revert(uint8_t *v, uint64_t n);

/* transform.cpp:241-279; out must hold ceil(4n/3)+4 bytes; returns output length */
uint64_t hco_rle_apply(const uint8_t *in, uint64_t n, uint8_t *out);
/* transform.cpp:281-292 + 137-159; returns decoded length (written only while < cap) */
uint64_t hco_rle_revert(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

/* transform.cpp:294-328 (+97-134, 66-94, 25-62, headers.cpp:18-63).
 * out must hold hco_adapt_bound(n, W) bytes. Returns 0 or 12; *out_len = header+data length;
 * *best_block = chosen block size. */
uint64_t hco_adapt_bound(uint64_t n, uint64_t width);
int hco_adapt_apply(const uint8_t *m, uint64_t width, uint64_t height, uint8_t *out,
                    uint64_t *out_len, uint64_t *best_block);
/* transform.cpp:330-361 (+162-216, headers.cpp:65-105). Allocates *out (free with hco_free).
 * Returns 0, 10, 11, 13, 14, 15, or 100 (forged block size 0; reference divides by zero) /
 * 101 (forged W*H too large to allocate; reference throws bad_alloc). */
int hco_adapt_revert(const uint8_t *in, uint64_t n, uint8_t **out, uint64_t *out_len);

/* FGK adaptive Huffman, faithful pointer-tree form with the pruned-DFS leader search
 * (huffman.cpp:23-217) driven like transform.cpp:363-406.
 * encode: bits written MSB-first into out (zero padded to a byte); returns bit count before
 * padding. out needs hco_fgk_bound(n) bytes. */
uint64_t hco_fgk_bound(uint64_t n);
uint64_t hco_fgk_encode(const uint8_t *sym, uint64_t n, uint8_t *out);
/* decode `count` symbols from nbits bits; returns 0 or 9 (bits exhausted) */
int hco_fgk_decode(const uint8_t *bits, uint64_t nbits, uint64_t count, uint8_t *sym);

/* Same coder in implicit slot form: the form the HIP kernels use.
 * Kept here so tests can show it equals the faithful form above. */
uint64_t hco_fgk_encode_slot(const uint8_t *sym, uint64_t n, uint8_t *out);
int hco_fgk_decode_slot(const uint8_t *bits, uint64_t nbits, uint64_t count, uint8_t *sym);

/* Whole pipeline = huffCompress (main.cpp:39-87) / huffDecompress (main.cpp:90-128).
 * Output is malloc'ed into *out (free with hco_free). compress status: 0, 4 (width 0),
 * 6 (size % width), 12; decompress: 0, 8, 9, 10, 11, 13, 14, 15, 100, 101. */
int hco_compress(const uint8_t *in, uint64_t n, int use_diff, int use_adapt, uint64_t width,
                 uint8_t **out, uint64_t *out_len);
int hco_decompress(const uint8_t *in, uint64_t n, uint8_t **out, uint64_t *out_len);
void hco_free(void *p);

/* Synthetic inputs of SURVEY.md Appendix D (kind 0 noise, 1 grad, 2 photo), stream k. */
void hco_synth(int kind, uint64_t k, uint64_t width, uint64_t height, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
