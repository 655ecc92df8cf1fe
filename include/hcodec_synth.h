/*
 * hcodec_synth.h — on-device synthetic 8-bit grayscale inputs for the
 * bench and the GPU tests. Not part of the reference's surface; it lets a batch be generated in
 * HBM with no host-to-device traffic. Byte-identical to oracle/hc_oracle.c:hco_synth.
 */
#ifndef HCODEC_SYNTH_H
#define HCODEC_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HC_SYNTH_NOISE 0
#define HC_SYNTH_GRAD 1
#define HC_SYNTH_PHOTO 2

/* Stream j (0 <= j < n_streams) = generator `kind`, index k0 + j, width x height bytes, written
 * to d_out + j * stride (device pointer). Asynchronous on `stream` (a hipStream_t). */
int hc_synth_batch(int kind, uint64_t k0, uint32_t n_streams, uint64_t width, uint64_t height,
                   uint8_t *d_out, uint64_t stride, void *stream);

#ifdef __cplusplus
}
#endif
#endif
