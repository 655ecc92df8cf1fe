// hc_synth.hip — SURVEY.md Appendix D generator on the device (bench / test inputs).
#include <hip/hip_runtime.h>

#include "hcodec.h"
#include "hcodec_synth.h"

namespace {

__device__ __forceinline__ uint64_t smix(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ int64_t floor_div4(int64_t a) { return a >= 0 ? a / 4 : -((-a + 3) / 4); }

// one thread per 4 output bytes of one row; grid.y = stream
__global__ void synth_kernel(int kind, uint64_t k0, uint64_t w, uint64_t h, uint8_t *out, uint64_t stride)
{
    const uint64_t k = k0 + blockIdx.y;
    const uint64_t s = 24301ull * 1000003ull + k;
    uint8_t *o = out + blockIdx.y * stride;
    const uint64_t n = w * h;
    const uint64_t T = 32;
    for (uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 4; i0 < n;
         i0 += (uint64_t)gridDim.x * blockDim.x * 4) {
        uint32_t word = 0;
        const uint32_t cnt = i0 + 4 <= n ? 4u : (uint32_t)(n - i0);
        for (uint32_t b = 0; b < cnt; ++b) {
            const uint64_t i = i0 + b, y = i / w, x = i % w;
            uint32_t v;
            if (kind == HC_SYNTH_NOISE) {
                v = (uint32_t)(smix(s, i) & 0xFF);
            } else if (kind == HC_SYNTH_GRAD) {
                v = (uint32_t)((x + 2 * y + k) & 0xFF);
            } else {
                const uint64_t t = (y / T) * (w / T) + x / T;
                const uint64_t th = smix(s ^ 0xABCDEF, t);
                const int64_t base = (int64_t)(th & 0xFF);
                const int64_t gx = (int64_t)((th >> 8) & 7) - 3;
                const int64_t gy = (int64_t)((th >> 11) & 7) - 3;
                const int64_t amp = (int64_t)((th >> 14) & 3);
                const bool flat = ((th >> 16) & 3) == 0;
                const int64_t nz = (int64_t)((smix(s, i) & 7) % (uint64_t)(2 * amp + 1)) - amp;
                if (flat) {
                    v = (uint32_t)base;
                } else {
                    const int64_t q = base + floor_div4((int64_t)(x % T) * gx + (int64_t)(y % T) * gy) + nz;
                    v = (uint32_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
                }
            }
            word |= v << (8 * b);
        }
        if (cnt == 4 && ((reinterpret_cast<uintptr_t>(o + i0) & 3) == 0)) {
            *reinterpret_cast<uint32_t *>(o + i0) = word;
        } else {
            for (uint32_t b = 0; b < cnt; ++b) o[i0 + b] = (uint8_t)(word >> (8 * b));
        }
    }
}

}  // namespace

extern "C" int hc_synth_batch(int kind, uint64_t k0, uint32_t n_streams, uint64_t width, uint64_t height,
                              uint8_t *d_out, uint64_t stride, void *stream)
{
    if (n_streams == 0 || width * height == 0) return HC_OK;
    if (!d_out || kind < 0 || kind > 2) return HC_ERR_ARG;
    const uint64_t n = width * height;
    uint64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    // grid.y (the stream) is limited to 65535: launch in chunks
    for (uint32_t s0 = 0; s0 < n_streams; s0 += 65535u) {
        const uint32_t cnt = n_streams - s0 < 65535u ? n_streams - s0 : 65535u;
        synth_kernel<<<dim3((unsigned)blocks, cnt), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
            kind, k0 + s0, width, height, d_out + s0 * stride, stride);
        if (hipGetLastError() != hipSuccess) return HC_ERR_DEVICE;
    }
    return HC_OK;
}
