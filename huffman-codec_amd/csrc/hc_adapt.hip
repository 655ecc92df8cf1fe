// hc_adapt.hip — adaptive block RLE (encode search + emit, decode) and the diff model on gfx950.
//
// Reference: transform.cpp:294-328 (block-size search), transform.cpp:97-134 (per-block
// horizontal / vertical choice), transform.cpp:66-94 + 25-62 (block scan geometry),
// headers.cpp:18-105 (adaptive header), transform.cpp:330-361 + 162-216 (revert),
// transform.cpp:220-239 (diff model).
//
// Encode: for every candidate block size B (8 .. 1024, <= W, <= H, <= 7 doublings) one
// workgroup per (block, scan order) folds the scan into a run summary (a monoid over byte
// runs whose closed-form MNP-5 cost, SURVEY.md Appendix A.3, gives the block's RLE length
// without emitting it); per-block min/argmin and the candidate's total follow; the host picks
// the first minimum; an exclusive scan of the chosen lengths places each block; one lane per
// block then emits its RLE bytes. Decode: one wavefront finds each block's start in the symbol
// stream (a wave scan of the revert machine's transition functions and of output lengths per
// 256 symbols), then one lane per block reverts and scatters in parallel; the diff revert is a
// parallel mod-256 scan.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "hc_internal.h"

namespace hc {
namespace {

// ------------------------------------------------------------------------- run summary ---

// MNP-5 bytes of a run of L equal bytes that is not the sequence's last run (closed form of
// transform.cpp:241-279): full 258-chunks cost 4, a remainder r costs r (r < 3) or 4.
__device__ __forceinline__ uint64_t run_cost(uint64_t L)
{
    const uint64_t r = L % 258;
    return 4 * (L / 258) + (r == 0 ? 0 : (r < 3 ? r : 4));
}
// the last run of a sequence: its final byte is always a literal (transform.cpp:252)
__device__ __forceinline__ uint64_t last_run_cost(uint64_t L) { return run_cost(L - 1) + 1; }

struct Runs {
    uint64_t n;    // bytes covered (0 = identity)
    uint64_t fa;   // length of the first run
    uint64_t lz;   // length of the last run
    uint64_t mid;  // cost of the runs strictly between the first and the last
    uint32_t a, z; // first and last byte
    uint32_t single;
};

__device__ __forceinline__ Runs runs_empty()
{
    Runs r;
    r.n = r.fa = r.lz = r.mid = 0;
    r.a = r.z = 0;
    r.single = 0;
    return r;
}

__device__ __forceinline__ void runs_push(Runs &r, uint32_t c)
{
    if (r.n == 0) {
        r.a = r.z = c;
        r.fa = r.lz = 1;
        r.single = 1;
        r.mid = 0;
    } else if (c == r.z) {
        ++r.lz;
        if (r.single) ++r.fa;
    } else {
        if (!r.single) r.mid += run_cost(r.lz);
        r.single = 0;
        r.z = c;
        r.lz = 1;
    }
    ++r.n;
}

__device__ __forceinline__ Runs runs_join(const Runs &x, const Runs &y)
{
    if (x.n == 0) return y;
    if (y.n == 0) return x;
    Runs r;
    r.n = x.n + y.n;
    r.a = x.a;
    r.z = y.z;
    if (x.z == y.a) {
        const uint64_t m = x.lz + y.fa;
        if (x.single && y.single) {
            r.single = 1;
            r.fa = r.lz = m;
            r.mid = 0;
        } else if (x.single) {
            r.single = 0;
            r.fa = m;
            r.lz = y.lz;
            r.mid = y.mid;
        } else if (y.single) {
            r.single = 0;
            r.fa = x.fa;
            r.lz = m;
            r.mid = x.mid;
        } else {
            r.single = 0;
            r.fa = x.fa;
            r.lz = y.lz;
            r.mid = x.mid + run_cost(m) + y.mid;
        }
    } else {
        r.single = 0;
        r.fa = x.fa;
        r.lz = y.lz;
        r.mid = (x.single ? 0 : x.mid + run_cost(x.lz)) + (y.single ? 0 : run_cost(y.fa) + y.mid);
    }
    return r;
}

__device__ __forceinline__ uint64_t runs_total(const Runs &r)
{
    if (r.n == 0) return 0;
    return r.single ? last_run_cost(r.fa) : run_cost(r.fa) + r.mid + last_run_cost(r.lz);
}

// transform.cpp:25-62
struct Geo {
    uint64_t x0, y0, sx, sy;
};
__device__ __forceinline__ Geo block_geo(uint64_t w, uint64_t h, uint64_t b, uint64_t i)
{
    const uint64_t per_row = (w + b - 1) / b;
    Geo g;
    g.x0 = (i % per_row) * b;
    g.y0 = (i / per_row) * b;
    g.sx = g.x0 + b > w ? w - g.x0 : b;
    g.sy = g.y0 + b > h ? h - g.y0 : b;
    return g;
}

constexpr int kCostThreads = 256;

// grid (blocks, 2): y = 0 horizontal scan, y = 1 vertical scan. Each thread folds a contiguous
// piece of the scan sequence; an ordered LDS tree joins the pieces.
__global__ __launch_bounds__(kCostThreads) void block_cost_kernel(const uint8_t *m, uint64_t w,
                                                                   uint64_t h, uint64_t b,
                                                                   uint64_t *cost)
{
    __shared__ Runs part[kCostThreads];
    const uint64_t blk = blockIdx.x;
    const bool horiz = blockIdx.y == 0;
    const Geo g = block_geo(w, h, b, blk);
    const uint64_t len = g.sx * g.sy;
    const uint64_t per = (len + blockDim.x - 1) / blockDim.x;
    const uint64_t beg = threadIdx.x * per;
    const uint64_t end = beg + per < len ? beg + per : len;
    Runs r = runs_empty();
    if (beg < end) {
        // transform.cpp:66-94: horizontal = row-major inside the block, vertical = column-major
        const uint64_t inner = horiz ? g.sx : g.sy;
        uint64_t o = beg / inner, q = beg % inner;  // outer / inner index of the scan
        for (uint64_t k = beg; k < end; ++k) {
            const uint64_t x = horiz ? q : o, y = horiz ? o : q;
            runs_push(r, m[(g.y0 + y) * w + g.x0 + x]);
            if (++q == inner) {
                q = 0;
                ++o;
            }
        }
    }
    part[threadIdx.x] = r;
    __syncthreads();
    for (unsigned s = 1; s < blockDim.x; s *= 2) {
        if ((threadIdx.x % (2 * s)) == 0 && threadIdx.x + s < blockDim.x)
            part[threadIdx.x] = runs_join(part[threadIdx.x], part[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) cost[blk * 2 + (horiz ? 0 : 1)] = runs_total(part[0]);
}

// transform.cpp:113-123: per block keep the shorter scan (tie -> horizontal); sum the data
__global__ void choose_kernel(const uint64_t *cost, uint64_t nb, uint64_t *len, uint8_t *dir,
                              unsigned long long *total)
{
    __shared__ unsigned long long acc[256];
    uint64_t sum = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nb;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t lh = cost[2 * i], lv = cost[2 * i + 1];
        const bool hz = lh <= lv;
        len[i] = hz ? lh : lv;
        dir[i] = hz ? 1 : 0;
        sum += hz ? lh : lv;
    }
    acc[threadIdx.x] = sum;
    __syncthreads();
    for (unsigned s = blockDim.x / 2; s > 0; s /= 2) {
        if (threadIdx.x < s) acc[threadIdx.x] += acc[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(total, acc[0]);
}

// headers.cpp:18-63: <u64 BE W><u64 BE H><u64 BE B><scan-direction bits, MSB first, 1 = h>
__global__ void header_kernel(uint8_t *out, uint64_t w, uint64_t h, uint64_t b, const uint8_t *dir,
                              uint64_t nb)
{
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < 24) {
        const uint64_t v = i < 8 ? w : (i < 16 ? h : b);
        out[i] = (uint8_t)(v >> (56 - 8 * (i % 8)));
    }
    const uint64_t nbytes = (nb + 7) / 8;
    if (i < nbytes) {
        uint32_t byte = 0;
        for (uint32_t k = 0; k < 8; ++k) {
            const uint64_t j = i * 8 + k;
            byte = (byte << 1) | (j < nb ? dir[j] : 0u);
        }
        out[24 + i] = (uint8_t)byte;
    }
}

// transform.cpp:241-279 on one block's scan, one lane per block
__global__ void emit_kernel(const uint8_t *m, uint64_t w, uint64_t h, uint64_t b, uint64_t nb,
                            const uint8_t *dir, const uint64_t *off, uint8_t *out)
{
    const uint64_t blk = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (blk >= nb) return;
    const Geo g = block_geo(w, h, b, blk);
    const bool horiz = dir[blk] != 0;
    const uint64_t len = g.sx * g.sy;
    const uint64_t inner = horiz ? g.sx : g.sy;
    uint8_t *o = out + off[blk];
    uint64_t p = 0, oo = 0, q = 0;
    uint32_t run_byte = 0, run = 0;
    for (uint64_t k = 0; k < len; ++k) {
        const uint64_t x = horiz ? q : oo, y = horiz ? oo : q;
        const uint32_t c = m[(g.y0 + y) * w + g.x0 + x];
        if (++q == inner) {
            q = 0;
            ++oo;
        }
        if (run != 0 && c == run_byte && k + 1 != len) {
            ++run;
            if (run <= 3) {
                o[p++] = (uint8_t)c;
            } else if (run == 258) {
                o[p++] = 255;
                run = 0;
            }
        } else {
            if (run >= 3) o[p++] = (uint8_t)(run - 3);
            o[p++] = (uint8_t)c;
            run_byte = c;
            run = 1;
        }
    }
}

// ------------------------------------------------------------------------------ decode ---

// Where each block's RLE data starts (transform.cpp:330-361 running revertRLEBlock,
// transform.cpp:162-187, block by block), reporting 13 / 14 / 15 exactly where the reference
// exits. One wavefront, 256 symbols per step (4 per lane). The revert machine's state r (0..3:
// how many equal literals precede; 3 = the next symbol is a count) moves by one of two functions
// per symbol — a literal repeating the previous symbol (r -> r + 1) or not (r -> 1), a count -> 0;
// from 0 both give 1, so the symbol before a block start never matters. A wave scan of their
// compositions gives each symbol's state, hence its output length (count: the symbol, literal:
// 1); a scan of lengths finds the first symbol where the block's byte count is reached. A block
// that ends inside the step re-scans the rest of the same registers from state 0.
constexpr uint32_t kFsmEq = 1u | 2u << 2 | 3u << 4;        // r: 0->1 1->2 2->3 3->0
constexpr uint32_t kFsmNe = 1u | 1u << 2 | 1u << 4;        // r: 0->1 1->1 2->1 3->0
constexpr uint32_t kFsmId = 0u | 1u << 2 | 2u << 4 | 3u << 6;

__device__ __forceinline__ uint32_t fsm_then(uint32_t g, uint32_t f)  // x -> g(f(x))
{
    uint32_t h = 0;
#pragma unroll
    for (uint32_t x = 0; x < 4; ++x) h |= ((g >> (2 * ((f >> (2 * x)) & 3u))) & 3u) << (2 * x);
    return h;
}

__global__ __launch_bounds__(64) void bounds_kernel(const uint8_t *sym, uint64_t nsym, uint64_t w,
                                                    uint64_t h, uint64_t b, uint64_t nb, uint64_t pos0,
                                                    uint64_t *start, int *status)
{
    const uint32_t lane = threadIdx.x;
    uint64_t pos = pos0;  // first symbol of the loaded step
    uint64_t blk = 0, got = 0;
    uint32_t r = 0, last = 0;  // machine state and previous symbol at the step's start
    if (lane == 0) start[0] = pos;
    uint64_t want = 0;
    if (nb) {
        const Geo g = block_geo(w, h, b, 0);
        want = g.sx * g.sy;
    }
    while (blk < nb) {
        const uint64_t avail = nsym - pos;
        const uint32_t m = avail < 256 ? (uint32_t)avail : 256u;
        if (m == 0) {  // transform.cpp:170-174: the block wants more, the stream is empty
            if (lane == 0) *status = HC_ERR_BLOCK_EOF;
            return;
        }
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) x[k] = 4 * lane + k < m ? sym[pos + 4 * lane + k] : 0u;
        const uint32_t up = __shfl_up(x[3], 1, 64);
        uint32_t lo = 0;  // symbols below lo belong to blocks already closed
        for (;;) {
            uint32_t f[4], F = kFsmId;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t i = 4 * lane + k;
                const uint32_t p = k ? x[k - 1] : (lane ? up : last);
                f[k] = (i >= lo && i < m) ? (x[k] == p ? kFsmEq : kFsmNe) : kFsmId;
                F = fsm_then(f[k], F);
            }
            uint32_t inc = F;
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t g = __shfl_up(inc, off, 64);
                inc = lane >= off ? fsm_then(inc, g) : inc;
            }
            const uint32_t ex = __shfl_up(inc, 1, 64);
            uint32_t s = ((lane ? ex : kFsmId) >> (2 * r)) & 3u;
            uint32_t len[4], tot = 0;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t i = 4 * lane + k;
                len[k] = (i >= lo && i < m) ? (s == 3 ? x[k] : 1u) : 0u;
                tot += len[k];
                s = (f[k] >> (2 * s)) & 3u;
            }
            uint32_t acc = tot;  // inclusive scan of lengths (<= 256 * 255)
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t g = __shfl_up(acc, off, 64);
                acc += lane >= off ? g : 0u;
            }
            const uint64_t need = want - got;  // >= 1
            const uint64_t hit = __ballot((uint64_t)acc >= need);
            if (!hit) {  // the block goes on past this step
                got += __shfl(acc, 63, 64);
                r = (__shfl(inc, 63, 64) >> (2 * r)) & 3u;
                const uint32_t lt = __shfl(x[(m - 1) & 3u], (m - 1) >> 2, 64);
                last = lt;
                pos += m;
                break;
            }
            // the first symbol whose running length reaches the block's size closes it
            const uint32_t L = (uint32_t)__builtin_ctzll(hit);
            uint32_t c = acc - tot, j = 0xFFFFFFFFu, cj = 0;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                c += len[k];
                if (j == 0xFFFFFFFFu && (uint64_t)c >= need) {
                    j = 4 * lane + k;
                    cj = c;
                }
            }
            j = __shfl(j, L, 64);
            cj = __shfl(cj, L, 64);
            if ((uint64_t)cj != need) {  // transform.cpp:178-182: a count overshoots the block
                if (lane == 0) *status = HC_ERR_BLOCK_DATA;
                return;
            }
            lo = j + 1;
            ++blk;
            if (lane == 0) start[blk] = pos + lo;
            if (blk == nb) {
                pos += lo;
                break;
            }
            const Geo g = block_geo(w, h, b, blk);
            want = g.sx * g.sy;
            got = 0;
            r = 0;
            if (lo == m) {
                pos += m;
                break;
            }
        }
    }
    // transform.cpp:354-358
    if (lane == 0) *status = pos != nsym ? HC_ERR_LEFTOVER : 0;
}

// transform.cpp:162-216 for one block per lane: revert its RLE and scatter in scan order
__global__ void unblock_kernel(const uint8_t *sym, uint64_t w, uint64_t h, uint64_t b,
                               uint64_t nb, const uint8_t *dirbits, const uint64_t *start,
                               uint8_t *m)
{
    const uint64_t blk = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (blk >= nb) return;
    const Geo g = block_geo(w, h, b, blk);
    const bool horiz = (dirbits[blk / 8] >> (7 - blk % 8)) & 1;
    const uint64_t inner = horiz ? g.sx : g.sy;
    const uint64_t want = g.sx * g.sy;
    uint64_t pos = start[blk], got = 0, oo = 0, q = 0;
    uint32_t run_byte = 0, run = 0;
    auto put = [&](uint32_t v) {
        const uint64_t x = horiz ? q : oo, y = horiz ? oo : q;
        m[(g.y0 + y) * w + g.x0 + x] = (uint8_t)v;
        if (++q == inner) {
            q = 0;
            ++oo;
        }
        ++got;
    };
    while (got < want) {
        const uint32_t c = sym[pos++];
        if (run == 3) {
            for (uint32_t r = 0; r < c; ++r) put(run_byte);
            run = 0;
        } else {
            put(c);
            if (c == run_byte) ++run;
            else {
                run_byte = c;
                run = 1;
            }
        }
    }
}

// transform.cpp:220-229, out of place
__global__ void diff_kernel(const uint8_t *in, uint8_t *out, uint64_t n)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint8_t)(in[i] - (i ? in[i - 1] : 0));
}

struct ByteAdd {
    __device__ __forceinline__ uint8_t operator()(uint8_t a, uint8_t b) const
    {
        return (uint8_t)(a + b);
    }
};

uint64_t ceil_div(uint64_t a, uint64_t b) { return a / b + (a % b != 0); }

#define HC_TRY(x)                          \
    do {                                   \
        hipError_t e_ = (x);               \
        if (e_ != hipSuccess) return e_;   \
    } while (0)

}  // namespace

hipError_t diff_apply(uint8_t *d, uint64_t n, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    uint8_t *tmp = nullptr;
    HC_TRY(hipMalloc((void **)&tmp, n));
    HC_TRY(hipMemcpyAsync(tmp, d, n, hipMemcpyDeviceToDevice, st));
    const uint64_t blocks = ceil_div(n, 256) < 8192 ? ceil_div(n, 256) : 8192;
    diff_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>(tmp, d, n);
    HC_TRY(hipGetLastError());
    return hipFree(tmp);
}

// transform.cpp:231-239: inclusive prefix sum mod 256
hipError_t diff_revert(uint8_t *d, uint64_t n, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    size_t tmp_bytes = 0;
    HC_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tmp_bytes, d, d, ByteAdd(), (int)n, st));
    void *tmp = nullptr;
    HC_TRY(hipMalloc(&tmp, tmp_bytes + 16));
    HC_TRY(hipcub::DeviceScan::InclusiveScan(tmp, tmp_bytes, d, d, ByteAdd(), (int)n, st));
    return hipFree(tmp);
}

hipError_t adapt_bound(uint64_t n, uint64_t width, uint64_t *bytes)
{
    (void)width;
    *bytes = 24 + n / 64 + 64 + n + n / 3 + n / 64 + 64;
    return hipSuccess;
}

// transform.cpp:294-328. Synchronous (the block-size choice is made on the host).
hipError_t adapt_encode(const uint8_t *m, uint64_t w, uint64_t h, uint8_t *out, uint64_t *d_out_len,
                        uint64_t *h_block, hipStream_t st)
{
    std::vector<uint64_t> sizes;
    for (uint64_t b = 8, step = 0; step <= 7 && b <= w && b <= h; ++step, b *= 2) sizes.push_back(b);
    const size_t nc = sizes.size();
    const uint64_t nb8 = ceil_div(w, 8) * ceil_div(h, 8);
    uint64_t *cost = nullptr, *len = nullptr, *off = nullptr;
    uint8_t *dir = nullptr;
    unsigned long long *total = nullptr;
    HC_TRY(hipMalloc((void **)&cost, nb8 * 2 * sizeof(uint64_t)));
    HC_TRY(hipMalloc((void **)&len, nb8 * sizeof(uint64_t)));
    HC_TRY(hipMalloc((void **)&off, (nb8 + 1) * sizeof(uint64_t)));
    HC_TRY(hipMalloc((void **)&dir, nb8));
    HC_TRY(hipMalloc((void **)&total, nc * sizeof(unsigned long long)));
    HC_TRY(hipMemsetAsync(total, 0, nc * sizeof(unsigned long long), st));
    for (size_t c = 0; c < nc; ++c) {
        const uint64_t b = sizes[c];
        const uint64_t nb = ceil_div(w, b) * ceil_div(h, b);
        block_cost_kernel<<<dim3((unsigned)nb, 2), dim3(b * b >= 4 * kCostThreads ? kCostThreads : 64), 0,
                            st>>>(m, w, h, b, cost);
        HC_TRY(hipGetLastError());
        const unsigned g = (unsigned)(ceil_div(nb, 256) < 1024 ? ceil_div(nb, 256) : 1024);
        choose_kernel<<<dim3(g), dim3(256), 0, st>>>(cost, nb, len, dir, total + c);
        HC_TRY(hipGetLastError());
    }
    std::vector<unsigned long long> tot(nc);
    HC_TRY(hipMemcpyAsync(tot.data(), total, nc * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HC_TRY(hipStreamSynchronize(st));
    // transform.cpp:309-325: first strictly smaller (header + data) wins
    size_t best = 0;
    uint64_t best_len = 0;
    for (size_t c = 0; c < nc; ++c) {
        const uint64_t nb = ceil_div(w, sizes[c]) * ceil_div(h, sizes[c]);
        const uint64_t l = 24 + ceil_div(nb, 8) + tot[c];
        if (c == 0 || l < best_len) {
            best = c;
            best_len = l;
        }
    }
    const uint64_t b = sizes[best];
    const uint64_t nb = ceil_div(w, b) * ceil_div(h, b);
    const uint64_t hdr = 24 + ceil_div(nb, 8);
    // re-derive the winner's per-block choice, then place and emit
    block_cost_kernel<<<dim3((unsigned)nb, 2), dim3(b * b >= 4 * kCostThreads ? kCostThreads : 64), 0, st>>>(
        m, w, h, b, cost);
    HC_TRY(hipGetLastError());
    {
        const unsigned g = (unsigned)(ceil_div(nb, 256) < 1024 ? ceil_div(nb, 256) : 1024);
        choose_kernel<<<dim3(g), dim3(256), 0, st>>>(cost, nb, len, dir, total);
        HC_TRY(hipGetLastError());
    }
    size_t tmp_bytes = 0;
    HC_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tmp_bytes, len, off, hipcub::Sum(), (uint64_t)hdr,
                                             (int)nb, st));
    void *tmp = nullptr;
    HC_TRY(hipMalloc(&tmp, tmp_bytes + 16));
    HC_TRY(hipcub::DeviceScan::ExclusiveScan(tmp, tmp_bytes, len, off, hipcub::Sum(), (uint64_t)hdr,
                                             (int)nb, st));
    header_kernel<<<dim3((unsigned)ceil_div(hdr, 256)), dim3(256), 0, st>>>(out, w, h, b, dir, nb);
    HC_TRY(hipGetLastError());
    emit_kernel<<<dim3((unsigned)ceil_div(nb, 64)), dim3(64), 0, st>>>(m, w, h, b, nb, dir, off, out);
    HC_TRY(hipGetLastError());
    HC_TRY(hipMemcpyAsync(d_out_len, &best_len, sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HC_TRY(hipFree(tmp));
    HC_TRY(hipFree(cost));
    HC_TRY(hipFree(len));
    HC_TRY(hipFree(off));
    HC_TRY(hipFree(dir));
    HC_TRY(hipFree(total));
    HC_TRY(hipStreamSynchronize(st));
    *h_block = b;
    return hipSuccess;
}

// transform.cpp:330-361 + headers.cpp:65-105. *d_matrix is allocated here (hipFree by caller).
hipError_t adapt_decode(const uint8_t *sym, uint64_t nsym, uint8_t **d_matrix, uint64_t *h_len,
                        int *h_status, hipStream_t st)
{
    *d_matrix = nullptr;
    *h_len = 0;
    if (nsym < 24) {  // headers.cpp:67-71
        *h_status = HC_ERR_ADAPT_HEADER;
        return hipSuccess;
    }
    uint8_t hdr[24];
    HC_TRY(hipMemcpyAsync(hdr, sym, 24, hipMemcpyDeviceToHost, st));
    HC_TRY(hipStreamSynchronize(st));
    uint64_t f[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 8; ++i) f[k] = (f[k] << 8) | hdr[8 * k + i];
    const uint64_t w = f[0], h = f[1], b = f[2];
    if (b == 0) {
        *h_status = HC_ERR_BLOCK_SIZE;
        return hipSuccess;
    }
    const uint64_t nb = ceil_div(w, b) * ceil_div(h, b);
    const uint64_t dir_bytes = ceil_div(nb, 8);
    if (nsym - 24 < dir_bytes) {  // headers.cpp:94-98
        *h_status = HC_ERR_ADAPT_DIRS;
        return hipSuccess;
    }
    if (w != 0 && h > (1ull << 36) / w) {
        *h_status = HC_ERR_TOO_LARGE;
        return hipSuccess;
    }
    const uint64_t n = w * h;
    uint8_t *m = nullptr;
    uint64_t *start = nullptr;
    int *dstat = nullptr;
    HC_TRY(hipMalloc((void **)&m, n + 16));
    HC_TRY(hipMalloc((void **)&start, (nb + 1) * sizeof(uint64_t)));
    HC_TRY(hipMalloc((void **)&dstat, sizeof(int)));
    bounds_kernel<<<1, 64, 0, st>>>(sym, nsym, w, h, b, nb, 24 + dir_bytes, start, dstat);
    HC_TRY(hipGetLastError());
    int status = 0;
    HC_TRY(hipMemcpyAsync(&status, dstat, sizeof(int), hipMemcpyDeviceToHost, st));
    HC_TRY(hipStreamSynchronize(st));
    if (status == 0 && nb) {
        unblock_kernel<<<dim3((unsigned)ceil_div(nb, 64)), dim3(64), 0, st>>>(sym, w, h, b, nb, sym + 24,
                                                                              start, m);
        HC_TRY(hipGetLastError());
    }
    HC_TRY(hipFree(start));
    HC_TRY(hipFree(dstat));
    HC_TRY(hipStreamSynchronize(st));
    if (status != 0) {
        (void)hipFree(m);
        *h_status = status;
        return hipSuccess;
    }
    *d_matrix = m;
    *h_len = n;
    *h_status = 0;
    return hipSuccess;
}

}  // namespace hc
