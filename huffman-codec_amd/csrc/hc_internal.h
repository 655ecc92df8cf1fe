// hc_internal.h — launchers shared between the kernel translation units and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hcodec.h"

namespace hc {

// One batch of independent streams. All pointers are device pointers.
struct Batch {
    const uint8_t *in;
    const uint64_t *in_offs;
    const uint64_t *in_lens;
    uint32_t n;
    uint8_t *out;
    const uint64_t *out_offs;
    const uint64_t *out_caps;
    uint64_t *out_lens;
    int32_t *status;
    uint32_t flags;  // header flags byte for SRC_SYMBOLS encodes
    uint32_t min_tree;  // set by the launchers: the smallest FGK tree layout (hc_debug_set_min_tree)
    uint32_t dec_small;  // set by launch_decode: 0 by payload rate, 1 / 2 every / no narrow stream small (hc_debug_set_dec_small)
};

enum EncSrc { SRC_RAW = 0, SRC_RAW_DIFF = 1, SRC_SYMBOLS = 2 };
enum DecDst { DST_RAW = 0, DST_SYMBOLS = 1 };

// Largest FGK symbol count the packed ("narrow") tree layout handles: weights live in 22 bits.
constexpr uint64_t kNarrowMaxSymbols = (1ull << 22) - 2;
// Largest count of the wide layout (32-bit weights, sentinel 0xFFFFFFFF).
constexpr uint64_t kWideMaxSymbols = 0xFFFFFFFFull - 1;

// fused [diff] -> RLE -> FGK encode, or FGK over a ready symbol stream (adaptive path)
hipError_t launch_encode(const Batch &b, EncSrc src, hipStream_t st, hipStream_t aux = nullptr);
// fused FGK decode -> RLE revert -> [diff revert] (diff taken from each stream's flags byte),
// or FGK decode to the symbol stream
hipError_t launch_decode(const Batch &b, DecDst dst, hipStream_t st);

// adaptive block RLE (hc_adapt.hip), batched: device pointers as in Batch, asynchronous on st.
// Encode: matrix i = in[in_offs[i] ..) of in_lens[i] bytes and width widths[i]; flags
// HC_FLAG_DIFF or 0; the whole -a stream (FGK included) lands in out. Decode: adaptive streams
// -> matrices (diff revert from each stream's flags byte). `work` (16-byte aligned) must hold
// the bound below; streams that do not fit report HC_ERR_CAPACITY.
hipError_t adapt_encode_batch(const Batch &b, const uint64_t *widths, void *work, uint64_t work_bytes,
                              hipStream_t st);
hipError_t adapt_decode_batch(const Batch &b, void *work, uint64_t work_bytes, hipStream_t st);
uint64_t adapt_encode_work_bound(uint64_t total_in, uint32_t n);
uint64_t adapt_decode_work_bound(uint64_t total_in, uint64_t total_out, uint32_t n);

// frees the host-batch pipeline slots' cached buffers (hc_release_cached; slots in use by a
// running call are left alone)
void pipe_release();

}  // namespace hc
