// hc_adapt.hip — adaptive block RLE on gfx950, batched: many W x H matrices per call.
//
// Reference: transform.cpp:294-328 (block-size search), transform.cpp:97-134 (per-block h / v
// choice), transform.cpp:25-94 (block geometry and scan order), headers.cpp:18-105 (adaptive
// header), transform.cpp:330-361 + 137-216 (revert), transform.cpp:220-239 (diff model),
// transform.cpp:241-279 (MNP-5 RLE). Model of the arithmetic: tests/adapt_cost_model.py.
//
// Encode (per batch, every kernel a persistent grid over a device-built work list):
//   plan      one workgroup: validate each matrix (4 / 6 / 12), count its tiles, candidate
//             block sizes, cost words and workspace slab; exclusive scans place everything.
//   tile      one workgroup per 128 x 128 tile: the tile (diff model applied on the fly) is
//             loaded once into LDS; 64-lane ballots turn it into "equal to the left / upper
//             neighbour" bit rows (Eh, Ev); every candidate B = 8..128 then costs every block
//             in both scan orders from those words: one block row (h) or column (v) per lane,
//             its first bit substituted by the comparison across the scan's row wrap, folded
//             by the run-segment monoid (no bytes emitted: the MNP-5 length is a closed form of
//             the runs) and joined across the block's lanes in order. Per
//             block one word (cost | h-flag) and per candidate one atomic total. For B >= 256
//             the tile also writes one 8-byte summary per tile row / column.
//   big       one workgroup per block of B >= 256: joins the tile summaries of its rows /
//             columns.
//   choose    one workgroup per matrix: first minimum of header + data over B
//             (transform.cpp:309-325), header + direction bits, exclusive scan of the winner's
//             block lengths in place.
//   emit      one wave per block: MNP-5 of the block's scan, 64 elements per step, from each
//             element's run offset (ballot of run starts, carried across steps); byte offsets
//             by ballot popcounts.
//   FGK       the batched FGK encoder over the symbol streams (hc_fgk.hip, SRC_SYMBOLS).
// Decode:
//   plan / FGK decode to symbols / parse headers (10, 11, 66, 67, capacity) / scan groups;
//   bounds    one wave per stream: where every K-th block starts (a wave scan of the revert
//             machine's transition functions and output lengths per 512 symbols, the next step's
//             dword loads in flight), reporting
//             13 / 14 / 15 where the reference exits;
//   unblock   one wave per group of K blocks (>= 1024 bytes): revert + scatter in scan order;
//   undiff    per 16 KB chunk: byte sums, a per-stream scan of them, byte prefix sums.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "hc_internal.h"

namespace hc {
namespace {

// Diagnostic build (-DHC_TC_PROF): tile_cost_kernel sums the s_memtime cycles of its phases
// (load, equality words, candidates, summaries) into g_tc_prof (hc_debug_tc_prof reads it).
// Slots 0-5: tile_cost (the tile_put barrier, its wait for the tile's loads, the rest of
// tile_put, equality words, candidates, summaries); 8-11: emit_tile (the same three, the emit).
#ifdef HC_TC_PROF
__device__ unsigned long long g_tc_prof[16];
#define HC_TC_BEGIN() uint64_t tc_t = __builtin_amdgcn_s_memtime()
#define HC_TC_MARK(i)                                                                              \
    do {                                                                                           \
        const uint64_t tc_n = __builtin_amdgcn_s_memtime();                                        \
        if (tid == 0) atomicAdd(&g_tc_prof[(i) - 1], (unsigned long long)(tc_n - tc_t));           \
        tc_t = tc_n;                                                                               \
    } while (0)
#else
#define HC_TC_BEGIN()
#define HC_TC_MARK(i)
#endif
// tile_put's phase marks (a no-op outside the HC_TC_PROF build)
struct NoMark {
    __device__ __forceinline__ void operator()(uint32_t) const {}
};

constexpr uint32_t kTile = 128;
constexpr uint32_t kCand = 8;        // B = 8 << c, c = 0..7 (transform.cpp:294-328, <= 7 doublings)
constexpr uint32_t kTileCand = 5;    // B <= 128: inside one tile
constexpr uint32_t kDS = 132;        // LDS row stride of a tile: 33 dwords, column reads conflict-free
constexpr uint32_t kGrid = 2048;     // persistent grids: workgroups
constexpr uint32_t kChunk = 16384;   // diff revert chunk
constexpr uint32_t kGroupBytes = 1024;

struct AMeta {
    uint64_t w, h;
    uint64_t cost0[kCand];           // encode: first cost word of candidate c
    unsigned long long total[kCand];  // encode: data bytes of candidate c
    uint64_t nbc[kCand];             // encode: blocks of candidate c
    uint64_t pieces;                 // encode: first tile-summary entry
    uint64_t offs;                   // encode: the winner's u64 block offsets (workspace offset)
    uint64_t slab;                   // first byte of the stream's workspace slab
    uint64_t sym;                    // first symbol byte (workspace offset)
    uint64_t starts;                 // decode: first group-start entry (workspace offset, bytes; mode 0: every block's)
    uint64_t csum;                   // decode: first chunk-sum byte (workspace offset)
    uint64_t nb, B, K, groups, chunks, hdr, count;
    uint32_t nc, diff;
    int32_t status;
    uint32_t best;                   // encode: the chosen candidate
    uint32_t mode;                   // decode: 0 tiles, one entry per block (B = 8..128, power of 2),
                                     // 1 one entry per block (B >= 256, power of 2), 2 K-block
                                     // groups (other B)
    uint32_t pad2;
    uint64_t tiles;                  // decode: tiles (mode 0)
    uint64_t ents;                   // decode: group-start entries reserved at `starts`
    // decode, parallel block-boundary pass (bounds_par: streams of >= kParMin block symbols)
    uint32_t pcap;                   // the slab holds the pass's data (dec_plan)
    uint32_t par;                    // the stream takes the pass (dec_header)
    uint32_t pfall;                  // par_scan gave up (a window past kWinCap): par_fix re-runs all
    uint32_t pad3;
    uint64_t psub, pchk, pz, pzi, ps0;  // workspace offsets: sub-chunk records, chunk records, Z, Z info, s0
    uint64_t nsub, nchk, preruns;
    uint64_t pdiag[8];               // debug build: par_scan cycle counts (scripts/par_diag.py)
};

// workspace: [meta n][idx0 n+1][idx1 n+1][idx2 n+1][idx3 n+1][sym_offs n][sym_lens n][sym_caps n]
//            [lens2 n][counters 16][slabs ...]
struct Ws {
    AMeta *meta;
    uint64_t *idx[4];
    uint64_t *sym_offs, *sym_lens, *sym_caps, *lens2;
    unsigned long long *ctr;
    uint8_t *base;       // the workspace itself (slab offsets are relative to it)
    uint64_t slab0, slab_end;
    uint32_t n;
};

__host__ __device__ inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
__host__ __device__ inline uint64_t cdiv(uint64_t a, uint64_t b) { return a / b + (a % b != 0); }

uint64_t ws_header(uint32_t n)
{
    return align_up((uint64_t)n * sizeof(AMeta), 256) + 4 * align_up(8ull * (n + 1), 256) +
           4 * align_up(8ull * n, 256) + 256;
}

Ws carve(void *work, uint64_t bytes, uint32_t n)
{
    Ws w;
    uint8_t *p = static_cast<uint8_t *>(work);
    uint64_t o = 0;
    w.base = p;
    w.n = n;
    w.meta = reinterpret_cast<AMeta *>(p + o);
    o += align_up((uint64_t)n * sizeof(AMeta), 256);
    for (int k = 0; k < 4; ++k) {
        w.idx[k] = reinterpret_cast<uint64_t *>(p + o);
        o += align_up(8ull * (n + 1), 256);
    }
    uint64_t **arr[4] = {&w.sym_offs, &w.sym_lens, &w.sym_caps, &w.lens2};
    for (int k = 0; k < 4; ++k) {
        *arr[k] = reinterpret_cast<uint64_t *>(p + o);
        o += align_up(8ull * n, 256);
    }
    w.ctr = reinterpret_cast<unsigned long long *>(p + o);
    o += 256;
    w.slab0 = o;
    w.slab_end = bytes;
    return w;
}

// --------------------------------------------------------------------- wave / WG helpers ---

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads and stores (__syncthreads' release fence would drain those too, so a tile
// prefetched into registers or cost words just stored would stall every barrier).
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// DPP data movement (gfx9 wave64): value of lane l - s within the 16-lane row (row_shr), of the
// row's lane 15 / the wave's lane 31 (row_bcast 15 / 31, rows picked by the row mask), of lane
// l - 1 across the wave (wave_shr 1). Lanes without a source get `id`.
template <int kCtrl, int kRows = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t id)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, kCtrl, kRows, 0xF, false);
}

// inclusive wave scan with an associative op(later, earlier) and its identity: rows by row_shr
// 1, 2, 4, 8, then rows 1 and 3 take lane 15 / 47, rows 2 and 3 lane 31 (no LDS traffic)
template <class Op>
__device__ __forceinline__ uint32_t wave_scan(uint32_t v, uint32_t id, Op op)
{
    v = op(v, dpp<0x111>(v, id));
    v = op(v, dpp<0x112>(v, id));
    v = op(v, dpp<0x114>(v, id));
    v = op(v, dpp<0x118>(v, id));
    v = op(v, dpp<0x142, 0xA>(v, id));
    v = op(v, dpp<0x143, 0xC>(v, id));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_incl(uint32_t v)
{
    return wave_scan(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t lane_shr1(uint32_t v, uint32_t id) { return dpp<0x138>(v, id); }
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// index i with pre[i] <= t < pre[i + 1] (pre[0] = 0, pre[n] = total, t < total)
// per: every item's count when they are all equal (the plan kernels store it in ctr[8 + column];
// ~0 otherwise): then a division replaces the binary search's dependent loads
__device__ __forceinline__ uint32_t find_item(const uint64_t *pre, uint32_t n, uint64_t t, uint64_t per)
{
    if (per != ~0ull && per != 0) return (uint32_t)(t / per);
    uint32_t lo = 0, hi = n;  // pre[lo] <= t < pre[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= t) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Exclusive scans of kC columns over n items in ONE workgroup of 1024 threads. need(i, v) fills
// the item's values; put(i, base) receives its exclusive prefix; tot[] the totals; uni[] each
// column's common value when every item has the same, else ~0 (find_item's fast path).
template <int kC, class Need, class Put>
__device__ void wg_scan(uint32_t n, Need need, Put put, uint64_t *tot, uint64_t *uni = nullptr)
{
    __shared__ uint64_t part[1024][kC];
    __shared__ uint32_t same[kC];
    const uint32_t t = threadIdx.x, per = (n + 1023) / 1024;
    const uint32_t b = t * per, e = b + per < n ? b + per : n;
    uint64_t s[kC], v0[kC];
    for (int c = 0; c < kC; ++c) s[c] = 0;
    if (t < kC) same[t] = 1;
    if (n) need(0, v0);
    __syncthreads();
    for (uint32_t i = b; i < e; ++i) {
        uint64_t v[kC];
        need(i, v);
        for (int c = 0; c < kC; ++c) {
            s[c] += v[c];
            if (v[c] != v0[c]) same[c] = 0;
        }
    }
    for (int c = 0; c < kC; ++c) part[t][c] = s[c];
    __syncthreads();
    if (uni && t < kC) uni[t] = (n && same[t]) ? v0[t] : ~0ull;
    if (t < kC) {  // one thread per column: sequential scan of 1024 partials
        uint64_t acc = 0;
        for (uint32_t k = 0; k < 1024; ++k) {
            const uint64_t v = part[k][t];
            part[k][t] = acc;
            acc += v;
        }
        tot[t] = acc;
    }
    __syncthreads();
    for (int c = 0; c < kC; ++c) s[c] = part[t][c];
    for (uint32_t i = b; i < e; ++i) {
        uint64_t v[kC];
        need(i, v);
        put(i, s);
        for (int c = 0; c < kC; ++c) s[c] += v[c];
    }
    __syncthreads();
}

// --------------------------------------------------------------- run-segment monoid ---
// A stretch of a block scan as a bit string (bit p = element p equals element p - 1):
// lead = ones before the first zero (= n if none), tail = ones after the last zero, mid = MNP-5
// bytes of the runs that start and end inside. tests/adapt_cost_model.py: Seg.

struct Seg {
    uint32_t n, lead, tail, mid;
};

__device__ __forceinline__ Seg seg_id()
{
    Seg s;
    s.n = s.lead = s.tail = s.mid = 0;
    return s;
}

// MNP-5 bytes of a run of L that is not the scan's last (closed form of transform.cpp:241-279)
__device__ __forceinline__ uint32_t run_cost(uint32_t L)
{
    const uint32_t q = L / 258u, r = L - q * 258u;
    return 4 * q + (r == 0 ? 0u : (r < 3 ? r : 4u));
}

// bits 0..n-1 of w, 1 <= n <= 64: every run strictly inside the word is < 64 long, so it
// costs 1, 2 or 4: a pattern count of zeros, 01 and 011 (read upwards)
__device__ __forceinline__ Seg seg_leaf(uint64_t w, uint32_t n)
{
    const uint64_t valid = n >= 64 ? ~0ull : ((1ull << n) - 1);
    w &= valid;
    const uint64_t z = ~w & valid;
    const uint32_t f = z ? (uint32_t)__builtin_ctzll(z) : 0u;
    const uint32_t l = z ? 63u - (uint32_t)__builtin_clzll(z) : 0u;
    const uint64_t m = ((1ull << l) - 1) & ~((1ull << f) - 1);
    Seg s;
    s.n = n;
    s.lead = z ? f : n;
    s.tail = z ? n - 1 - l : 0u;
    s.mid = __popcll(z & m) + __popcll(w & (z << 1) & m) + 2 * __popcll(w & (w << 1) & (z << 2) & m);
    return s;
}

__device__ __forceinline__ Seg seg_join(const Seg &x, const Seg &y)
{
    const bool x0 = x.lead < x.n, y0 = y.lead < y.n;
    Seg r;
    r.n = x.n + y.n;
    if (!y0) {
        r.lead = x0 ? x.lead : x.n + y.n;
        r.tail = x0 ? x.tail + y.n : 0u;
        r.mid = x.mid;
    } else if (!x0) {
        r.lead = x.n + y.lead;
        r.tail = y.tail;
        r.mid = y.mid;
    } else {
        r.lead = x.lead;
        r.tail = y.tail;
        r.mid = x.mid + run_cost(x.tail + 1 + y.lead) + y.mid;
    }
    return r;
}

// cost of a whole block scan (its first bit is 0: the block starts a run)
__device__ __forceinline__ uint32_t seg_cost(const Seg &s) { return s.n ? s.mid + run_cost(s.tail) + 1 : 0u; }

template <int kCtrl>
__device__ __forceinline__ Seg seg_dpp(const Seg &s)
{
    Seg r;
    r.n = dpp<kCtrl>(s.n, 0u);
    r.lead = dpp<kCtrl>(s.lead, 0u);
    r.tail = dpp<kCtrl>(s.tail, 0u);
    r.mid = dpp<kCtrl>(s.mid, 0u);
    return r;
}

// the Seg of lane l + d (d a power of two): DPP row_shl inside 16-lane rows, else a permute
__device__ __forceinline__ Seg seg_shfl_down(const Seg &s, uint32_t d)
{
    switch (d) {
    case 1: return seg_dpp<0x101>(s);
    case 2: return seg_dpp<0x102>(s);
    case 4: return seg_dpp<0x104>(s);
    case 8: return seg_dpp<0x108>(s);
    default: {
        Seg r;
        r.n = __shfl_down(s.n, d, 64);
        r.lead = __shfl_down(s.lead, d, 64);
        r.tail = __shfl_down(s.tail, d, 64);
        r.mid = __shfl_down(s.mid, d, 64);
        return r;
    }
    }
}

// ordered join over aligned groups of g lanes (g a power of two <= 64); lane 0 of a group ends
// with the group's fold
__device__ __forceinline__ Seg seg_group(Seg s, uint32_t g, uint32_t lane)
{
    for (uint32_t st = 1; st < g; st <<= 1) {
        const Seg t = seg_shfl_down(s, st);
        if ((lane & (2 * st - 1)) == 0) s = seg_join(s, t);
    }
    return s;
}

// a block row / column: bits [off, off + n) of a 128-bit tile row, bit 0 replaced by `first`
__device__ __forceinline__ Seg seg_piece(const uint64_t *w, uint32_t off, uint32_t n, uint32_t first)
{
    if (n <= 64) {
        const uint64_t v = ((w[off >> 6] >> (off & 63)) & ~1ull) | first;
        return seg_leaf(v, n);
    }
    return seg_join(seg_leaf((w[0] & ~1ull) | first, 64), seg_leaf(w[1], n - 64));
}

// 8-byte tile summary of a tile row / column for the blocks of B >= 256: the segment of bits
// 1..len-1 (lead, tail: <= 127; mid <= 170), bit 0, the first and the last value
__device__ __forceinline__ uint64_t piece_pack(const Seg &s, uint32_t e0, uint32_t first, uint32_t last)
{
    return (uint64_t)s.lead | (uint64_t)s.tail << 8 | (uint64_t)s.mid << 16 | (uint64_t)first << 32 |
           (uint64_t)last << 40 | (uint64_t)e0 << 48;
}
__device__ __forceinline__ Seg piece_seg(uint64_t p, uint32_t n)
{
    Seg s;
    s.n = n;
    s.lead = p & 0xFF;
    s.tail = (p >> 8) & 0xFF;
    s.mid = (p >> 16) & 0xFFFF;
    return s;
}

// --------------------------------------------------------------------------- encode ------

struct EncArgs {
    const uint8_t *in;
    const uint64_t *in_offs, *in_lens, *widths;
    uint32_t n, diff;
};

// blocks of size b in a w x h matrix (transform.cpp:410-418)
__host__ __device__ inline uint64_t nblocks(uint64_t w, uint64_t h, uint64_t b) { return cdiv(w, b) * cdiv(h, b); }

__global__ __launch_bounds__(1024) void enc_plan_kernel(EncArgs a, Ws ws)
{
    auto need = [&](uint32_t i, uint64_t *v) {
        const uint64_t len = a.in_lens[i], w = a.widths[i];
        const uint64_t h = w ? len / w : 0;
        const bool ok = w != 0 && len % w == 0 && w >= 8 && h >= 8;
        uint64_t cost = 0, big = 0;
        uint32_t nc = 0;
        for (uint64_t b = 8, c = 0; ok && c < kCand && b <= w && b <= h; ++c, b *= 2, ++nc) {
            cost += nblocks(w, h, b);
            if (c >= kTileCand) big += nblocks(w, h, b);
        }
        const uint64_t ntx = cdiv(w, kTile), nty = cdiv(h, kTile);
        const uint64_t pieces = (ok && nc > kTileCand) ? h * ntx + w * nty : 0;
        const uint64_t nb8 = ok ? nblocks(w, h, 8) : 0;
        // MNP-5 of a block of L bytes <= 4L/3 + 1, header 24 + one bit per block
        const uint64_t syms = ok ? len + len / 3 + nb8 + nb8 / 8 + 64 : 0;
        v[0] = ok ? ntx * nty : 0;
        v[1] = big;
        v[2] = nb8;
        v[3] = ok ? align_up(4 * cost, 16) + align_up(8 * pieces, 16) + align_up(8 * nb8, 16) + align_up(syms, 16) : 0;
    };
    auto put = [&](uint32_t i, const uint64_t *base) {
        uint64_t v[4];
        need(i, v);
        AMeta &m = ws.meta[i];
        const uint64_t len = a.in_lens[i], w = a.widths[i];
        const uint64_t h = w ? len / w : 0;
        m.w = w;
        m.h = h;
        m.diff = a.diff;
        // main.cpp:195-199 (width 0), main.cpp:54-58 (size not a multiple of the width),
        // transform.cpp:300-304 (either side < 8)
        m.status = w == 0 ? HC_ERR_WIDTH : (len % w ? HC_ERR_MATRIX_SIZE : (w < 8 || h < 8 ? HC_ERR_DIMS : 0));
        m.slab = ws.slab0 + base[3];
        if (m.status == 0 && m.slab + v[3] > ws.slab_end) m.status = HC_ERR_CAPACITY;
        uint64_t o = m.slab, nc = 0;
        for (uint64_t b = 8, c = 0; c < kCand; ++c, b *= 2) {
            m.total[c] = 0;
            const bool on = m.status == 0 && b <= w && b <= h;
            m.nbc[c] = on ? nblocks(w, h, b) : 0;
            m.cost0[c] = o;  // a byte offset into the workspace
            o += 4 * m.nbc[c];
            nc += on;
        }
        m.nc = (uint32_t)nc;
        o = align_up(o, 16);
        m.pieces = o;
        o += align_up(v[3] ? 8 * (nc > kTileCand ? h * cdiv(w, kTile) + w * cdiv(h, kTile) : 0) : 0, 16);
        m.offs = o;  // one u64 per block of the winner (at most the B = 8 count)
        o += align_up(v[3] ? 8 * v[2] : 0, 16);
        m.sym = o;
        ws.sym_offs[i] = o;
        ws.sym_lens[i] = 0;
        ws.idx[0][i] = base[0];
        ws.idx[1][i] = base[1];
        ws.idx[2][i] = base[2];
    };
    __shared__ uint64_t tot[4], uni[4];
    wg_scan<4>(a.n, need, put, tot, uni);
    if (threadIdx.x == 0) {
        for (int k = 0; k < 3; ++k) {
            ws.idx[k][a.n] = tot[k];
            ws.ctr[k] = tot[k];
            ws.ctr[8 + k] = uni[k];
        }
    }
}

template <class T>
__device__ __forceinline__ T *at(const Ws &ws, uint64_t off)
{
    return reinterpret_cast<T *>(ws.base + off);
}

// LDS image of a tile: row r <-> y = ty0 + r - 1 (row 0: the row above the tile), byte c <->
// x = tx0 + c - 4 (c = 3: the column left of the tile), rows kDS bytes apart.
#define DT(r, xl) D[(r) * kDS + (xl) + 4]

// one unaligned dword of the stream at byte lin (bytes outside [0, n) read as 0)
__device__ __forceinline__ uint32_t load4(const uint8_t *m, int64_t lin, uint64_t n)
{
    typedef uint32_t u32u __attribute__((aligned(1)));
    if (lin >= 0 && (uint64_t)lin + 4 <= n) return *reinterpret_cast<const u32u *>(m + lin);
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k)
        if (lin + k >= 0 && (uint64_t)(lin + k) < n) v |= (uint32_t)m[lin + k] << (8 * k);
    return v;
}

// 0x80 in every byte of x that is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x)
{
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// bit q (0..3): byte q of a equals byte q of b (the four flags gathered by one multiply)
__device__ __forceinline__ uint32_t eq_nibble(uint32_t a, uint32_t b)
{
    return (((zero_bytes(a ^ b) >> 7) * 0x204081u) >> 21) & 0xFu;
}

// bytewise a - b and a + b (mod 256 per byte)
__device__ __forceinline__ uint32_t sub8(uint32_t a, uint32_t b)
{
    return ((a | 0x80808080u) - (b & 0x7F7F7F7Fu)) ^ ((a ^ ~b) & 0x80808080u);
}
__device__ __forceinline__ uint32_t add8(uint32_t a, uint32_t b)
{
    return ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
}

// (row, dword) of the items tid, tid + 256, tid + 512, ... of a tile image nd dwords wide,
// stepped without a division per item
struct TileWalk {
    uint32_t r, d, q, rem, nd;
    __device__ __forceinline__ TileWalk(uint32_t nd_, uint32_t tid) : nd(nd_)
    {
        r = tid / nd;
        d = tid - r * nd;
        q = 256 / nd;
        rem = 256 - q * nd;
    }
    __device__ __forceinline__ void next()
    {
        d += rem;
        r += q;
        if (d >= nd) {
            d -= nd;
            ++r;
        }
    }
};

// The tile a persistent workgroup's loop index u stands for. Workgroups are dealt round-robin
// over the 8 XCDs (each with its own L2): in each round of G = gridDim.x tiles, the workgroups
// of one XCD (b, b + 8, ..) take a contiguous run of G / 8 tiles, so a tile and its left /
// right neighbours -- whose loads share the 128-byte lines at the tile's edges, and the row
// above -- mostly meet in one L2 (the identity in a last, partial round).
#ifndef HC_XCD
#define HC_XCD 1
#endif
__device__ __forceinline__ uint64_t xcd_tile(uint64_t u, uint64_t G, uint64_t n)
{
    const uint64_t r = u / G, b = u - r * G, base = r * G;
    if (!HC_XCD || (G & 7) || base + G > n) return u;
    return base + (b & 7) * (G >> 3) + (b >> 3);
}

// The thread index, made opaque at the top of each pass of a persistent tile loop: the LDS
// addresses derived from it are then recomputed where they are used instead of hoisted out of
// the loop, where the hoisted set did not fit the registers and was spilled to scratch memory
// (tile_cost: 59 VGPRs spilled, 3.8 -> 3.1 ms on A512 without them).
#ifndef HC_LAUNDER
#define HC_LAUNDER 1
#endif
__device__ __forceinline__ uint32_t tid_here()
{
    uint32_t t = threadIdx.x;
#if HC_LAUNDER
    asm volatile("" : "+v"(t));
#endif
    return t;
}

// A tile of the work list (one workgroup's unit in tile_cost / emit_tile): its matrix and place.
struct TileAt {
    uint32_t i;            // matrix
    bool ok;               // the matrix is valid (status 0)
    uint64_t W, H, tx0, ty0, n;
    uint32_t tw, th;
    const uint8_t *mat;
};
__device__ __forceinline__ TileAt tile_at(const EncArgs &a, const Ws &ws, uint64_t t)
{
    TileAt g;
    g.i = find_item(ws.idx[0], a.n, t, ws.ctr[8 + 0]);
    const AMeta &M = ws.meta[g.i];
    g.ok = M.status == 0;
    g.W = M.w;
    g.H = M.h;
    g.n = M.w * M.h;
    const uint64_t ntx = cdiv(g.W, kTile), local = t - ws.idx[0][g.i];
    g.tx0 = (local % ntx) * kTile;
    g.ty0 = (local / ntx) * kTile;
    g.tw = (uint32_t)(g.W - g.tx0 < kTile ? g.W - g.tx0 : kTile);
    g.th = (uint32_t)(g.H - g.ty0 < kTile ? g.H - g.ty0 : kTile);
    g.mat = a.in + a.in_offs[g.i];
    return g;
}

// The LDS image of a tile: rows ty0 - 1 .. ty0 + th - 1, bytes tx0 - 4 .. tx0 + tw - 1 (DT),
// diff model applied (transform.cpp:220-229: d[k] = m[k] - m[k-1] over the linear matrix,
// m[-1] = 0). Built in two halves, so that a workgroup fetches its next tile into registers while
// it works on the current one: tile_fetch issues the raw dword loads (coalesced along each row;
// one aligned load per dword when the rows are dword-aligned, as in every 512-wide batch), one
// item per thread and u ((kTile + 8) / 4 dwords x (kTile + 1) rows <= kLU x 256); tile_put
// applies the diff model in registers and stores them (each dword's previous byte is the top
// byte of the item before it, the dword before in the row image; a row's first dword takes a
// stray one, harmless: only its byte 3, x = tx0 - 1, is ever read, and that needs just its own
// byte 2).
constexpr uint32_t kLU = ((kTile + 1) * ((kTile + 8) / 4) + 255) / 256;
__device__ __forceinline__ void tile_fetch(const TileAt &g, uint32_t *v, uint32_t tid)
{
    const uint32_t nd = (g.tw + 7) / 4, items = (g.th + 1) * nd;
    const bool aligned = ((reinterpret_cast<uintptr_t>(g.mat) | g.W) & 3) == 0;
    if (aligned && g.ty0 > 0 && (g.ty0 + g.th - 1) * g.W + g.tx0 + 4 * nd - 4 <= g.n) {
        // (uniform) every item inside the matrix: one pointer per thread, stepped q rows and
        // rem dwords per item (one row more when the dword index wraps)
        const uint32_t q = 256 / nd, rem = 256 - q * nd;
        uint32_t d = tid % nd;
        const uint8_t *p = g.mat + ((g.ty0 + tid / nd - 1) * g.W + g.tx0 - 4 + 4 * d);
        const uint64_t step = q * g.W + 4 * rem, wrap = g.W - 4 * nd;
#pragma unroll
        for (uint32_t u = 0; u < kLU; ++u) {
            v[u] = u * 256 + tid < items ? *reinterpret_cast<const uint32_t *>(p) : 0u;
            d += rem;
            p += step;
            if (d >= nd) {
                d -= nd;
                p += wrap;
            }
        }
        return;
    }
    TileWalk wk(nd, tid);
#pragma unroll
    for (uint32_t u = 0; u < kLU; ++u, wk.next()) {
        const uint32_t it = u * 256 + tid;
        const uint32_t r = wk.r, d = wk.d;
        const int64_t lin = (int64_t)(g.ty0 + r) * (int64_t)g.W - (int64_t)g.W + (int64_t)g.tx0 - 4 + 4 * (int64_t)d;
        const bool on = it < items && (r > 0 || g.ty0 > 0);
        const bool whole = on && aligned && lin >= 0 && (uint64_t)lin + 4 <= g.n;
        v[u] = whole ? *reinterpret_cast<const uint32_t *>(g.mat + lin) : (on ? load4(g.mat, lin, g.n) : 0u);
    }
}
template <class Mark = NoMark>
__device__ __forceinline__ void tile_put(uint8_t *D, uint32_t *edge, const TileAt &g, uint32_t *v, bool diff,
                                         uint32_t tid, Mark mark = {})
{
    const uint32_t nd = (g.tw + 7) / 4, items = (g.th + 1) * nd;
    const uint32_t lane = tid & 63, wv = tid >> 6;
    // the first barrier also ends the previous tile: no thread writes D before all have
    // finished reading it (tile_cost_kernel has no barrier at the end of a tile)
    if (diff) {
        // the previous item's dword is lane - 1's (wave_shr 1); a wave's lane 0 takes it from the
        // lane 63 before it through edge[] (item u * 256 + tid - 1)
        if (lane == 63) {
#pragma unroll
            for (uint32_t u = 0; u < kLU; ++u) edge[4 * u + wv] = v[u];
        }
    }
    lds_barrier();
    mark(0);
#ifdef HC_TC_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mark(1);
#endif
    if (diff) {
#pragma unroll
        for (uint32_t u = 0; u < kLU; ++u) {
            uint32_t pv = lane_shr1(v[u], 0u);
            if (lane == 0) pv = wv ? edge[4 * u + wv - 1] : (u ? edge[4 * u - 1] : 0u);
            v[u] = sub8(v[u], (v[u] << 8) | (pv >> 24));
        }
    }
    // LDS byte kDS r + 4 d of item (r, d), stepped like tile_fetch's pointer
    const uint32_t q = 256 / nd, rem = 256 - q * nd, step = q * kDS + 4 * rem, wrap = kDS - 4 * nd;
    uint32_t d = tid % nd, at = (tid / nd) * kDS + 4 * d;
#pragma unroll
    for (uint32_t u = 0; u < kLU; ++u) {
        if (u * 256 + tid < items) *reinterpret_cast<uint32_t *>(D + at) = v[u];
        d += rem;
        at += step;
        if (d >= nd) {
            d -= nd;
            at += wrap;
        }
    }
    lds_barrier();
    mark(2);
}

// the value of lane l + d (d a power of two): DPP row_shl inside 16-lane rows, else a permute
__device__ __forceinline__ uint32_t shl_down(uint32_t v, uint32_t d)
{
    switch (d) {
    case 1: return dpp<0x101>(v, 0u);
    case 2: return dpp<0x102>(v, 0u);
    case 4: return dpp<0x104>(v, 0u);
    case 8: return dpp<0x108>(v, 0u);
    default: return __shfl_down(v, d, 64);
    }
}

// llvm.amdgcn.writelane (no clang builtin in this toolchain; bound by name as in hc_fgk.hip)
extern "C" __device__ int amdgcn_writelane(int x, int l, int v) __asm("llvm.amdgcn.writelane.i32");

// Whole 128 x 128 tiles, B <= 64: the first bit of every block line's scan (transform.cpp:66-94:
// the comparison across the scan's line wrap, 0 on a block's first line), as 128-bit masks over
// the tile's lines, per candidate c and block column (h) / block row (v) b:
// WM[o][32 - (32 >> c) + b] (31 per order). One wave per order and half of the lines (lane =
// line): the 16 first and 16 last values of its 8-wide steps give all 31 comparisons.
__device__ __forceinline__ void wrap_masks(const uint8_t *D, uint64_t *WM, uint32_t wv, uint32_t lane)
{
    const uint32_t o = wv >> 1, half = wv & 1, line = 64 * half + lane;
    // h: DT(y + 1, 8k), DT(y, 8k + 7); v: DT(8k + 1, x), DT(8k + 8, x - 1)
    const uint8_t *fp = D + (o ? kDS + 4 + line : (line + 1) * kDS + 4);
    const uint8_t *lp = D + (o ? 8 * kDS + 3 + line : line * kDS + 11);
    const uint32_t st = o ? 8 * kDS : 8u;
    uint32_t mlo = 0, mhi = 0;  // lane i: mask i
    auto put = [&](uint32_t i, bool eq, uint32_t B) __attribute__((always_inline)) {
        const uint64_t m = ballot(eq && (line & (B - 1)) != 0);
        mlo = (uint32_t)amdgcn_writelane((int)(uint32_t)m, (int)i, (int)mlo);
        mhi = (uint32_t)amdgcn_writelane((int)(uint32_t)(m >> 32), (int)i, (int)mhi);
    };
    // two halves of 8 steps (B <= 64 pairs stay inside one), 16 values live at a time
    uint32_t f0 = 0;
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        uint32_t f[8], l[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            f[k] = fp[(8 * h + k) * st];
            l[k] = lp[(8 * h + k) * st];
        }
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) {
            const uint32_t s = 1u << c;  // B / 8
#pragma unroll
            for (uint32_t b = 0; b < (8u >> c); ++b)
                put(32 - (32 >> c) + (8u >> c) * h + b, f[b * s] == l[b * s + s - 1], 8 * s);
        }
        if (h == 0) f0 = f[0];
        else put(30, f0 == l[7], 128);
    }
    if (lane < 31) WM[(o * 32 + lane) * 2 + half] = (uint64_t)mhi << 32 | mlo;
}

// Whole 128 x 128 tiles, B = 8 << c <= 64: the (h, v) cost of every block into hv. One 64-bit
// word of a block's scan per thread and order (64 / B block lines from 8-, 16-, 32- or 64-bit
// reads of the Eh / Ev rows, first bits from WM); v blocks are taken column-major so a wave's
// lanes read few distinct words. The MNP-5 length is a pattern count over the scan (a run of L
// costs 1 + [L >= 2] + 2 [L >= 3], counted at its first element with a two-bit look-ahead into
// the next word), summed over the block's lanes, plus the last run's rule (run_cost(L - 1) + 1,
// from the block's last zero bit) — exact while no run reaches 259 elements, which needs an
// all-ones word; a wave holding one (B >= 32) folds the run-segment monoid instead.
template <uint32_t c>
__device__ __forceinline__ void fast_cost(const uint64_t *E, const uint64_t *WM, uint32_t *hv, uint32_t tid,
                                          uint32_t lane)
{
    constexpr uint32_t B = 8u << c, lg = 3 + c;
    constexpr uint32_t lnb = 7 - lg;       // log2 blocks per tile side
    constexpr uint32_t lwpb = 2 * lg - 6;  // log2 words per block
    constexpr uint32_t G = 1u << lwpb;
    constexpr uint32_t lpw = 64 >> lg;  // block lines per word
    constexpr uint64_t FM = c == 0 ? 0x0101010101010101ull : c == 1 ? 0x0001000100010001ull : c == 2 ? 0x0000000100000001ull : 1ull;
    const uint8_t *Eb = reinterpret_cast<const uint8_t *>(E);
    const uint8_t *Mb = reinterpret_cast<const uint8_t *>(WM);
    const uint32_t blk = tid >> lwpb, j = tid & (G - 1);
    const uint32_t bmin = blk & ((1u << lnb) - 1), bmaj = blk >> lnb;
#pragma unroll
    for (uint32_t o = 0; o < 2; ++o) {
        const uint32_t bx = o ? bmaj : bmin, by = o ? bmin : bmaj;
        const uint32_t l0 = ((o ? bx : by) << lg) + j * lpw, c0 = (o ? by : bx) << lg;
        const uint8_t *rp = Eb + o * 16 * kTile + l0 * 16 + (c0 >> 3);
        uint64_t word = 0;
#pragma unroll
        for (uint32_t q = 0; q < lpw; ++q) {
            uint64_t v;
            if constexpr (c == 0) v = rp[16 * q];
            else if constexpr (c == 1) v = *reinterpret_cast<const uint16_t *>(rp + 16 * q);
            else if constexpr (c == 2) v = *reinterpret_cast<const uint32_t *>(rp + 16 * q);
            else v = *reinterpret_cast<const uint64_t *>(rp + 16 * q);
            word |= v << (q * B);
        }
        const uint32_t mb = (uint32_t)(Mb[(o * 32 + 32 - (32 >> c) + (o ? by : bx)) * 16 + (l0 >> 3)] >> (l0 & 7)) &
                            ((1u << lpw) - 1);
        uint64_t first;
        if constexpr (c == 0) {
            first = (uint64_t)(((mb >> 4) * 0x204081u) & 0x01010101u) << 32 | (((mb & 15u) * 0x204081u) & 0x01010101u);
        } else if constexpr (c == 1) {
            first = (uint64_t)(((mb >> 2) & 1u) | ((mb & 8u) << 13)) << 32 | ((mb & 1u) | ((mb & 2u) << 15));
        } else if constexpr (c == 2) {
            first = (uint64_t)(mb >> 1) << 32 | (mb & 1u);
        } else {
            first = mb;
        }
        word = (word & ~FM) | first;
        // the next word of the block's scan (lane + 1), none after the block's last
        uint32_t nx = 0;
        if constexpr (G > 1) {
            nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)word, 0x130, 0xF, 0xF, true);  // wave_shl 1
            nx = j == G - 1 ? 0u : nx;
        }
        const uint64_t Z = ~word;
        const uint64_t A = Z & ((word >> 1) | (uint64_t)(nx & 1u) << 63);
        const uint64_t C = A & ((word >> 2) | (uint64_t)(nx & 3u) << 62);
        uint32_t s = (uint32_t)(__popcll(Z) + __popcll(A) + 2 * __popcll(C));
        uint32_t lz = Z ? j * 64 + 63 - (uint32_t)__builtin_clzll(Z) : 0u;  // the last zero bit (bit 0 is one)
#pragma unroll
        for (uint32_t st = 1; st < G; st <<= 1) {
            const uint32_t s2 = shl_down(s, st), z2 = shl_down(lz, st);
            s += s2;
            lz = lz > z2 ? lz : z2;
        }
        uint32_t cost;
        if (c >= 2 && ballot(Z == 0)) {  // a run may reach 259: the monoid (wave-uniform)
            cost = seg_cost(seg_group(seg_leaf(word, 64), G, lane));
        } else {
            const uint32_t Lm = B * B - lz;  // the last run: run_cost(Lm - 1) + 1 for the counted g(Lm)
            cost = s + (Lm >= 4 ? 1u : 0u) - (Lm == 3 ? 1u : 0u);
        }
        if (j == 0) hv[(o << (2 * lnb)) + (by << lnb) + bx] = cost;
    }
}

// Whole tiles, B = 128 (one block per order): fast_cost's pattern count over the 256 words of
// each order, one per thread (word j = half j & 1 of line j >> 1; the look-ahead reads the low
// byte of word j + 1 itself, since it may sit in the next wave). Per wave and order: the count,
// the last zero bit and whether a word is all ones, into st[o][wave] (the caller joins them).
__device__ __forceinline__ void stats128(const uint64_t *E, const uint64_t *WM, uint32_t (*st)[4][3], uint32_t tid,
                                         uint32_t lane, uint32_t wv)
{
    const uint8_t *Mb = reinterpret_cast<const uint8_t *>(WM);
    const uint8_t *Eb = reinterpret_cast<const uint8_t *>(E);
    auto wrap = [&](uint32_t o, uint32_t r) __attribute__((always_inline)) {
        return (uint32_t)(Mb[(o * 32 + 30) * 16 + (r >> 3)] >> (r & 7)) & 1u;
    };
#pragma unroll
    for (uint32_t o = 0; o < 2; ++o) {
        const uint32_t j = tid;
        uint64_t word = E[o * 2 * kTile + j];
        if ((j & 1) == 0) word = (word & ~1ull) | wrap(o, j >> 1);
        uint32_t nx = 0;
        if (j < 2 * kTile - 1) {
            nx = Eb[(o * 2 * kTile + j + 1) * 8];
            if ((j & 1) == 1) nx = (nx & ~1u) | wrap(o, (j + 1) >> 1);
        }
        const uint64_t Z = ~word;
        const uint64_t A = Z & ((word >> 1) | (uint64_t)(nx & 1u) << 63);
        const uint64_t C = A & ((word >> 2) | (uint64_t)(nx & 3u) << 62);
        const uint32_t s = (uint32_t)(__popcll(Z) + __popcll(A) + 2 * __popcll(C));
        const uint32_t lz = Z ? j * 64 + 63 - (uint32_t)__builtin_clzll(Z) : 0u;
        const uint32_t sw = readlane(wave_sum_incl(s), 63);
        const uint32_t zw = readlane(wave_scan(lz, 0u, [](uint32_t x, uint32_t y) { return x > y ? x : y; }), 63);
        const bool ones = ballot(Z == 0) != 0;
        if (lane == 0) {
            st[o][wv][0] = sw;
            st[o][wv][1] = zw;
            st[o][wv][2] = ones;
        }
    }
}

// transform.cpp:97-134 / 294-328 (every candidate block's h / v scan length) for B <= 128, one
// workgroup per 128 x 128 tile of the work list (persistent grid): 1. the tile image in LDS
// (tile_put; the next tile's loads in flight meanwhile), 2. the Eh / Ev equality words (and the
// wrap masks of a whole tile), 3. every candidate's block costs (fast_cost / stats128 on whole
// tiles, the run-segment monoid on partial ones) into the cost words and per-candidate totals,
// 4. the tile row / column summaries the blocks of B >= 256 are joined from (big_cost_kernel).
#ifndef HC_TC_WPE
#define HC_TC_WPE 5
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HC_TC_WPE))) void tile_cost_kernel(EncArgs a, Ws ws)
{
    __shared__ uint8_t D[(kTile + 1) * kDS];  // DT(r, xl): y = ty0 + r - 1, x = tx0 + xl
    __shared__ uint64_t E[4 * kTile];         // Eh[r][2] then Ev[c][2]
    __shared__ uint32_t hv[2][2][256];        // candidate c's block costs, h / v: hv[c & 1]
    __shared__ Seg part[8];
    __shared__ uint64_t WM[2 * 32 * 2];       // wrap_masks (whole tiles)
    __shared__ uint32_t st128[2][4][3];       // stats128
    __shared__ uint32_t HV[682];              // whole tiles: every candidate's block costs (h then v)
    __shared__ uint32_t edge[4 * kLU];        // tile_put
    const uint32_t tid = threadIdx.x;  // (lane and wave: per tile, tid_here)
    const uint64_t ntiles = ws.ctr[0];
    const bool diff = a.diff != 0;
    // the next tile's raw dwords are in flight while this one is worked on
    uint32_t v[kLU];
    TileAt nx;
    if (blockIdx.x < ntiles) {
        nx = tile_at(a, ws, xcd_tile(blockIdx.x, gridDim.x, ntiles));
        if (nx.ok) tile_fetch(nx, v, tid);
    }
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tid = tid_here(), lane = tid & 63, wv = tid >> 6;  // (tid_here)
        const TileAt g = nx;
        const uint32_t i = g.i;
        AMeta &M = ws.meta[i];
        // read once, before the tile's atomics (after them the compiler must reload from memory)
        const uint32_t nc = M.nc;
        const uint64_t pieces = M.pieces;
        HC_TC_BEGIN();
        // 1. the tile plus one row above and one column to the left, diff model applied
#ifdef HC_TC_PROF
        if (g.ok) tile_put(D, edge, g, v, diff, tid, [&](uint32_t k) { HC_TC_MARK(k + 1); });
#else
        if (g.ok) tile_put(D, edge, g, v, diff, tid);
#endif
        if (t + gridDim.x < ntiles) {
            nx = tile_at(a, ws, xcd_tile(t + gridDim.x, gridDim.x, ntiles));
            if (nx.ok) tile_fetch(nx, v, tid);
        }
        if (!g.ok) continue;  // (uniform over the workgroup)
        const uint64_t W = g.W, H = g.H, tx0 = g.tx0, ty0 = g.ty0;
        const uint64_t ntx = cdiv(W, kTile);
        const uint32_t tw = g.tw, th = g.th;
        const bool whole = tw == kTile && th == kTile;
        // 2. Eh[r][k] bit j: x = tx0 + 64k + j equals x - 1 (row ty0 + r); Ev[c][k] bit j: y = ty0 +
        //    64k + j equals y - 1 (column tx0 + c). Eh: one word per thread from 16 dwords of its row
        //    (SWAR equality nibbles); Ev: lane = row, 4 ballots per dword column.
        {
            const uint32_t r = tid >> 1, k = tid & 1;
            uint64_t word = 0;
            if (r < th) {
                const uint8_t *row = D + (r + 1) * kDS + 4 + 64 * k;  // DT(r + 1, 64 k)
                uint32_t prev = *reinterpret_cast<const uint32_t *>(row - 4);
                uint32_t lo = 0, hi = 0;
#pragma unroll
                for (uint32_t m = 0; m < 16; ++m) {
                    const uint32_t w = *reinterpret_cast<const uint32_t *>(row + 4 * m);
                    const uint32_t nib = eq_nibble(w, (w << 8) | (prev >> 24));
                    if (m < 8) lo |= nib << (4 * m);
                    else hi |= nib << (4 * (m - 8));
                    prev = w;
                }
                word = (uint64_t)hi << 32 | lo;
                const uint32_t valid = tw > 64 * k ? tw - 64 * k : 0u;  // columns inside the tile
                word &= valid >= 64 ? ~0ull : ((1ull << valid) - 1);
                if (tx0 == 0 && k == 0) word &= ~1ull;  // x = 0 has no left neighbour
            }
            E[2 * r + k] = word;
            // Ev by SWAR down the columns: thread = 4 columns (dword c4) x 16 rows (rb); per row one
            // dword compare against the row above, its 4 byte flags shifted into 4 row masks, which
            // land as 16-bit pieces of the columns' Ev words. (Before: lane = row, a ballot and a
            // select per column -- ~500 VALU per wave and tile against ~210; A512 tile_cost 3.19 /
            // 3.10 -> 2.88 / 2.98 ms, scripts/tile_exp.py, outputs identical.)
            {
                const uint32_t c4 = tid & 31, rb = tid >> 5;
                uint32_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
                const uint8_t *col = D + 4 + 4 * c4;
#pragma unroll 4
                for (uint32_t rr = 0; rr < 16; ++rr) {
                    const uint32_t y = 16 * rb + rr;
                    const uint32_t a = *reinterpret_cast<const uint32_t *>(col + (y + 1) * kDS);
                    const uint32_t b = *reinterpret_cast<const uint32_t *>(col + y * kDS);
                    const uint32_t z = y < th && ty0 + y > 0 ? zero_bytes(a ^ b) : 0u;
                    acc0 |= ((z >> 7) & 1u) << rr;
                    acc1 |= ((z >> 15) & 1u) << rr;
                    acc2 |= ((z >> 23) & 1u) << rr;
                    acc3 |= ((z >> 31) & 1u) << rr;
                }
                uint16_t *ev = reinterpret_cast<uint16_t *>(E + 2 * kTile);  // column c: words 2 c, 2 c + 1
                const uint32_t c = 4 * c4, piece = 4 * (rb >> 2) + (rb & 3);
                ev[8 * c + piece] = (uint16_t)(c < tw ? acc0 : 0u);
                ev[8 * (c + 1) + piece] = (uint16_t)(c + 1 < tw ? acc1 : 0u);
                ev[8 * (c + 2) + piece] = (uint16_t)(c + 2 < tw ? acc2 : 0u);
                ev[8 * (c + 3) + piece] = (uint16_t)(c + 3 < tw ? acc3 : 0u);
            }
            if (whole) wrap_masks(D, WM, wv, lane);
        }
        lds_barrier();
        // (Eh / Ev by index into E, never as a selected pointer: a select of the two became a
        // scratch-memory pointer table and flat loads)
        constexpr uint32_t kEv = 2 * kTile;
        HC_TC_MARK(4);
        // 3. blocks of B <= 128, both scan orders
        //    (one copy per candidate: B, the lines per word and the group sizes are constants, so
        //    each thread's LDS reads unroll and issue together)
        const uint32_t nct = nc < kTileCand ? nc : kTileCand;
        uint32_t tot[kTileCand] = {};  // this thread's share of each candidate's total
        auto candidate = [&](auto cc) __attribute__((always_inline)) {
            constexpr uint32_t c = decltype(cc)::value;
            uint32_t(*hx)[256] = hv[c & 1];  // double-buffered: one barrier per candidate
            constexpr uint32_t B = 8u << c, lg = 3 + c;
            const uint32_t nbx = (tw + B - 1) >> lg, nby = (th + B - 1) >> lg;
            const uint32_t per_o = (nbx * nby) << lg, items = 2 * per_o;
            const bool full = (tw & (B - 1)) == 0 && (th & (B - 1)) == 0;
            // whole blocks: one 64-element word of the block's scan per lane (64 / B block rows or
            // columns, B = 128: half of one), first bits substituted, so a block of B = 8 is one
            // leaf and no join; 2 (h, v) x tw x th / 64 items
            constexpr uint32_t lwpb = lg <= 3 ? 0u : 2 * lg - 6;  // log2 of the words per block
            const uint32_t nwords = (tw * th) >> 6;
            for (uint32_t base = 0; full && base < 2 * nwords; base += 256) {
                const uint32_t it = base + tid;
                const uint32_t o = it >= nwords, wi = it - (o ? nwords : 0u);
                const uint32_t blk = wi >> lwpb, j = wi & ((1u << lwpb) - 1);
                const uint32_t bx = blk % nbx, by = blk / nbx;
                const uint32_t x0 = bx << lg, y0 = by << lg;
                uint64_t word = 0;
                if (it < 2 * nwords) {
                    const uint32_t e2 = o ? kEv : 0u;
                    const uint32_t l0 = o ? x0 : y0, c0 = o ? y0 : x0;  // first line, offset in it
                    if constexpr (B <= 64) {
                        constexpr uint32_t lpw = 64 >> lg;
                        const uint32_t r0 = j * lpw;
                        constexpr uint64_t msk = B >= 64 ? ~0ull : (1ull << (B & 63)) - 1;
#pragma unroll
                        for (uint32_t q = 0; q < lpw; ++q) {
                            const uint32_t r = r0 + q;
                            uint64_t bits = (E[e2 + 2 * (l0 + r) + (c0 >> 6)] >> (c0 & 63)) & msk & ~1ull;
                            if (r) {  // the scan's step across the line wrap (transform.cpp:66-94)
                                const bool eq = o ? DT(y0 + 1, x0 + r) == DT(y0 + B, (int)(x0 + r) - 1)
                                                  : DT(y0 + r + 1, x0) == DT(y0 + r, x0 + B - 1);
                                bits |= eq;
                            }
                            word |= bits << ((q * B) & 63);
                        }
                    } else {  // B = 128 (x0 = y0 = 0): word j = half j & 1 of line j >> 1
                        const uint32_t r = j >> 1;
                        word = E[e2 + 2 * r + (j & 1)];
                        if ((j & 1) == 0) {
                            word &= ~1ull;
                            if (r) word |= o ? DT(1, r) == DT(B, (int)r - 1) : DT(r + 1, 0) == DT(r, B - 1);
                        }
                    }
                }
                Seg sg = it < 2 * nwords ? seg_leaf(word, 64) : seg_id();
                const uint32_t G = 1u << lwpb;
                sg = seg_group(sg, G < 64 ? G : 64u, lane);
                if (G <= 64) {
                    if ((lane & (G - 1)) == 0 && it < 2 * nwords) hx[o][blk] = seg_cost(sg);
                } else if (lane == 0) {
                    part[4 * o + wv] = sg;
                }
            }
            for (uint32_t base = 0; !full && base < items; base += 256) {
                const uint32_t it = base + tid;
                const uint32_t o = it >= per_o, q = it - (o ? per_o : 0u);
                const uint32_t blk = q >> lg, r = q & (B - 1);
                const uint32_t bx = blk % nbx, by = blk / nbx;
                const uint32_t x0 = bx << lg, y0 = by << lg;
                const uint32_t sx = tw - x0 < B ? tw - x0 : B, sy = th - y0 < B ? th - y0 : B;
                Seg s = seg_id();
                if (it < items) {
                    if (o == 0 && r < sy) {  // block row r (transform.cpp:66-94, horizontal)
                        const uint32_t y = y0 + r;
                        const uint32_t first =
                            r ? (uint32_t)(DT(y + 1, x0) == DT(y, x0 + sx - 1)) : 0u;
                        s = seg_piece(E + 2 * y, x0, sx, first);
                    } else if (o == 1 && r < sx) {  // block column r (vertical)
                        const uint32_t x = x0 + r;
                        const uint32_t first =
                            r ? (uint32_t)(DT(y0 + 1, x) == DT(y0 + sy, (int)x - 1)) : 0u;
                        s = seg_piece(E + kEv + 2 * x, y0, sy, first);
                    }
                }
                s = seg_group(s, B < 64 ? B : 64u, lane);
                if (B <= 64) {
                    if ((lane & (B - 1)) == 0 && it < items) hx[o][blk] = seg_cost(s);
                } else if (lane == 0) {
                    part[wv] = s;
                }
            }
            lds_barrier();
            if constexpr (B == 128) {
                if (tid < 2)
                    hx[tid][0] = full ? seg_cost(seg_join(seg_join(part[4 * tid], part[4 * tid + 1]),
                                                          seg_join(part[4 * tid + 2], part[4 * tid + 3])))
                                      : seg_cost(seg_join(part[2 * tid], part[2 * tid + 1]));
                lds_barrier();
            }
            // transform.cpp:113-123: the shorter scan, ties horizontal; word = cost | h << 31
            const uint32_t nblk = nbx * nby;
            const uint64_t per_row = cdiv(W, B);
            uint32_t sum = 0;
            for (uint32_t b = tid; b < nblk; b += 256) {
                const uint32_t hc = hx[0][b], vc = hx[1][b];
                const uint64_t gi = (ty0 / B + b / nbx) * per_row + tx0 / B + b % nbx;
                at<uint32_t>(ws, M.cost0[c])[gi] = hc <= vc ? (hc | 0x80000000u) : vc;
                sum += hc <= vc ? hc : vc;
            }
            tot[c] += sum;
        };
        if (whole && nct == kTileCand) {
            // whole tiles: every candidate's block costs at once (one barrier), B = 128 from the
            // per-wave counts unless a word is all ones
            // (sched_barrier: one candidate's registers at a time; the prefetch holds 18)
            fast_cost<0>(E, WM, HV, tid, lane);
            __builtin_amdgcn_sched_barrier(0);
            fast_cost<1>(E, WM, HV + 512, tid, lane);
            __builtin_amdgcn_sched_barrier(0);
            fast_cost<2>(E, WM, HV + 640, tid, lane);
            __builtin_amdgcn_sched_barrier(0);
            fast_cost<3>(E, WM, HV + 672, tid, lane);
            __builtin_amdgcn_sched_barrier(0);
            stats128(E, WM, st128, tid, lane, wv);
            lds_barrier();
            uint32_t ones = 0;
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) ones |= st128[k >> 2][k & 3][2];
            // transform.cpp:113-123: the shorter scan, ties horizontal; word = cost | h << 31
            auto put = [&](uint32_t c, uint32_t lnb, uint32_t off, uint32_t b, uint32_t hc, uint32_t vc)
                __attribute__((always_inline)) {
                    const uint32_t B = 8u << c;
                    const uint64_t gi = (ty0 / B + (b >> lnb)) * cdiv(W, B) + tx0 / B + (b & ((1u << lnb) - 1));
                    at<uint32_t>(ws, M.cost0[c])[gi] = hc <= vc ? (hc | 0x80000000u) : vc;
                    tot[c] += hc <= vc ? hc : vc;
                    (void)off;
                };
            put(0, 4, 0, tid, HV[tid], HV[256 + tid]);
            if (tid < 64) {
                put(1, 3, 512, tid, HV[512 + tid], HV[576 + tid]);
            } else if (tid < 80) {
                put(2, 2, 640, tid - 64, HV[640 + tid - 64], HV[656 + tid - 64]);
            } else if (tid < 84) {
                put(3, 1, 672, tid - 80, HV[672 + tid - 80], HV[676 + tid - 80]);
            } else if (tid < 85 && !ones) {
                uint32_t hv2[2];
#pragma unroll
                for (uint32_t o = 0; o < 2; ++o) {
                    const uint32_t S = st128[o][0][0] + st128[o][1][0] + st128[o][2][0] + st128[o][3][0];
                    const uint32_t z = max(max(st128[o][0][1], st128[o][1][1]), max(st128[o][2][1], st128[o][3][1]));
                    const uint32_t Lm = kTile * kTile - z;
                    hv2[o] = S + (Lm >= 4 ? 1u : 0u) - (Lm == 3 ? 1u : 0u);
                }
                put(4, 0, 680, 0, hv2[0], hv2[1]);
            }
            if (ones) candidate(std::integral_constant<uint32_t, 4>{});  // (uniform)
        } else {
            if (nct > 0) candidate(std::integral_constant<uint32_t, 0>{});
            if (nct > 1) candidate(std::integral_constant<uint32_t, 1>{});
            if (nct > 2) candidate(std::integral_constant<uint32_t, 2>{});
            if (nct > 3) candidate(std::integral_constant<uint32_t, 3>{});
            if (nct > 4) candidate(std::integral_constant<uint32_t, 4>{});
        }
        // the candidates' totals: one atomic per wave and candidate
#pragma unroll
        for (uint32_t c = 0; c < kTileCand; ++c) {
            const uint32_t w = readlane(wave_sum_incl(tot[c]), 63);
            if (lane == 0 && c < nct) atomicAdd(&M.total[c], (unsigned long long)w);
        }
        HC_TC_MARK(5);
        // 4. tile summaries for the blocks of B >= 256
        if (nc > kTileCand) {
            const uint64_t nty = cdiv(H, kTile);
            uint64_t *pc = at<uint64_t>(ws, pieces);
            if (tid < th) {
                const uint64_t *w = E + 2 * tid;
                const Seg s = tw > 1 ? (tw > 64 ? seg_join(seg_leaf(w[0] >> 1, 63), seg_leaf(w[1], tw - 64))
                                                : seg_leaf(w[0] >> 1, tw - 1))
                                     : seg_id();
                pc[(ty0 + tid) * ntx + tx0 / kTile] =
                    piece_pack(s, (uint32_t)(w[0] & 1), DT(tid + 1, 0), DT(tid + 1, tw - 1));
            } else if (tid >= 128 && tid - 128 < tw) {
                const uint32_t x = tid - 128;
                const uint64_t *w = E + kEv + 2 * x;
                const Seg s = th > 1 ? (th > 64 ? seg_join(seg_leaf(w[0] >> 1, 63), seg_leaf(w[1], th - 64))
                                                : seg_leaf(w[0] >> 1, th - 1))
                                     : seg_id();
                pc[H * ntx + (tx0 + x) * nty + ty0 / kTile] =
                    piece_pack(s, (uint32_t)(w[0] & 1), DT(1, x), DT(th, x));
            }
        }
        HC_TC_MARK(6);  // (the next tile_put's first barrier ends this tile)
    }
}

// ordered join of one Seg per thread over a 256-thread workgroup (thread 0 gets the fold)
__device__ __forceinline__ Seg seg_block(Seg s, Seg *part, uint32_t tid)
{
    s = seg_group(s, 64, tid & 63);
    if ((tid & 63) == 0) part[tid >> 6] = s;
    lds_barrier();
    Seg r = seg_id();
    if (tid == 0) r = seg_join(seg_join(part[0], part[1]), seg_join(part[2], part[3]));
    lds_barrier();
    return r;
}

// blocks of B >= 256: rows (h) / columns (v) joined from the tile summaries
__global__ __launch_bounds__(256) void big_cost_kernel(EncArgs a, Ws ws)
{
    __shared__ Seg part[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t items = ws.ctr[1];
    for (uint64_t t = blockIdx.x; t < items; t += gridDim.x) {
        const uint32_t i = find_item(ws.idx[1], a.n, t, ws.ctr[8 + 1]);
        AMeta &M = ws.meta[i];
        if (M.status) continue;
        uint64_t k = t - ws.idx[1][i];
        uint32_t c = kTileCand;
        while (c < kCand - 1 && k >= M.nbc[c]) k -= M.nbc[c++];
        const uint64_t W = M.w, H = M.h, B = 8ull << c;
        const uint64_t ntx = cdiv(W, kTile), nty = cdiv(H, kTile), per_row = cdiv(W, B);
        const uint64_t x0 = (k % per_row) * B, y0 = (k / per_row) * B;
        const uint64_t sx = W - x0 < B ? W - x0 : B, sy = H - y0 < B ? H - y0 : B;
        const uint64_t *pc = at<uint64_t>(ws, M.pieces);
        uint32_t cost[2];
        for (uint32_t o = 0; o < 2; ++o) {
            // o = 0: rows y0.. of width sx over tiles x0/128..; o = 1: columns
            const uint64_t lines = o ? sx : sy, first_line = o ? x0 : y0;
            const uint64_t t0 = (o ? y0 : x0) / kTile, t1 = ((o ? y0 + sy : x0 + sx) - 1) / kTile;
            const uint64_t span = o ? H : W;
            const uint64_t stride = o ? nty : ntx;
            const uint64_t *P = pc + (o ? H * ntx : 0);
            const uint64_t per = (lines + 255) / 256;
            const uint64_t lb = tid * per, le = lb + per < lines ? lb + per : lines;
            Seg acc = seg_id();
            for (uint64_t r = lb; r < le; ++r) {
                const uint64_t line = first_line + r;
                const uint32_t prev_last = r ? (uint32_t)(P[(line - 1) * stride + t1] >> 40) & 0xFF : 0u;
                for (uint64_t tt = t0; tt <= t1; ++tt) {
                    const uint64_t e = P[line * stride + tt];
                    const uint64_t len = span - tt * kTile < kTile ? span - tt * kTile : kTile;
                    const uint32_t b0 = tt == t0 ? (r ? (uint32_t)(((e >> 32) & 0xFF) == prev_last) : 0u)
                                                 : (uint32_t)(e >> 48) & 1u;
                    acc = seg_join(acc, seg_join(seg_leaf(b0, 1), piece_seg(e, (uint32_t)len - 1)));
                }
            }
            cost[o] = seg_cost(seg_block(acc, part, tid));
        }
        if (tid == 0) {
            const uint32_t hc = cost[0], vc = cost[1];
            at<uint32_t>(ws, M.cost0[c])[k] = hc <= vc ? (hc | 0x80000000u) : vc;
            atomicAdd(&M.total[c], (unsigned long long)(hc <= vc ? hc : vc));
        }
    }
}

// transform.cpp:309-325 (first minimum of header + data), headers.cpp:18-63 (header), then the
// winner's block lengths -> their offsets, in place
__global__ __launch_bounds__(256) void choose_kernel(EncArgs a, Ws ws)
{
    __shared__ uint64_t part[256];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        AMeta &M = ws.meta[i];
        if (M.status) {
            if (tid == 0) ws.sym_lens[i] = 0;
            continue;
        }
        uint32_t best = 0;
        uint64_t best_len = 0;
        for (uint32_t c = 0; c < M.nc; ++c) {
            const uint64_t l = 24 + cdiv(M.nbc[c], 8) + M.total[c];
            if (c == 0 || l < best_len) {
                best = c;
                best_len = l;
            }
        }
        const uint64_t nb = M.nbc[best], B = 8ull << best, hdr = 24 + cdiv(nb, 8);
        uint8_t *sym = at<uint8_t>(ws, M.sym);
        uint32_t *wd = at<uint32_t>(ws, M.cost0[best]);
        if (tid < 24) {
            const uint64_t v = tid < 8 ? M.w : (tid < 16 ? M.h : B);
            sym[tid] = (uint8_t)(v >> (56 - 8 * (tid % 8)));
        }
        for (uint64_t k = tid; k < hdr - 24; k += 256) {  // direction bits, MSB first, 1 = h
            uint32_t byte = 0;
            for (uint32_t j = 0; j < 8; ++j) {
                const uint64_t b = 8 * k + j;
                byte = byte << 1 | (b < nb ? wd[b] >> 31 : 0u);
            }
            sym[24 + k] = (uint8_t)byte;
        }
        __syncthreads();
        // exclusive scan of the chosen lengths into the u64 block offsets
        const uint64_t per = (nb + 255) / 256, lb = tid * per, le = lb + per < nb ? lb + per : nb;
        uint64_t s = 0;
        for (uint64_t k = lb; k < le; ++k) s += wd[k] & 0x7FFFFFFFu;
        part[tid] = s;
        __syncthreads();
        if (tid == 0) {
            uint64_t acc = 0;
            for (uint32_t k = 0; k < 256; ++k) {
                const uint64_t v = part[k];
                part[k] = acc;
                acc += v;
            }
        }
        __syncthreads();
        s = part[tid];
        uint64_t *offs = at<uint64_t>(ws, M.offs);
        for (uint64_t k = lb; k < le; ++k) {
            offs[k] = s;
            s += wd[k] & 0x7FFFFFFFu;
        }
        if (tid == 0) {
            M.nb = nb;
            M.B = B;
            M.best = best;
            M.hdr = hdr;
            M.count = best_len;
            ws.sym_lens[i] = M.status ? 0 : best_len;
        }
        __syncthreads();
    }
}

// q / d for q < 2^24 (block-relative positions of the encoder: blocks <= 1024 x 1024)
__device__ __forceinline__ uint32_t div_small(uint32_t q, uint32_t d, float inv)
{
    uint32_t r = (uint32_t)((float)q * inv);
    r -= r * d > q;
    r += (r + 1) * d <= q;
    return r;
}

// transform.cpp:241-279 on one block's scan, by one wave, 64 elements per step (model:
// tests/adapt_cost_model.py emit_lanes): element p's run offset o comes from a ballot of run
// starts (carried across steps), j = o mod 258; it emits its byte for j <= 2, 255 at j = 257,
// the count j - 2 where its run ends (3 <= j + 1 <= 257), and the block's last element is a
// literal. Byte offsets: popcounts of two ballots. value(p) = the p-th element in scan order.
// o mod 258 for o < 516 (run offsets: at most the previous step's offset mod 258 plus 258;
// v_mul_hi_u32 and v_mul_lo_u32 of a division by the constant issue at a quarter of the rate)
__device__ __forceinline__ uint32_t mod258(uint32_t o) { return o >= 258u ? o - 258u : o; }

template <class Value>
__device__ __forceinline__ void emit_block(Value value, uint32_t L, uint8_t *out, uint32_t lane)
{
    const uint64_t lt = lanes_below(lane);
    uint32_t pv = 0, po = 0;  // value and run offset of the previous step's last element
    uint64_t q = 0;           // bytes written
    // each step's elements are read one step ahead (lanes past the block read its last element)
    uint32_t v = value(lane < L ? lane : L - 1);
    for (uint32_t base = 0; base < L; base += 64) {
        const uint32_t p = base + lane;
        const bool valid = p < L;
        const uint32_t pn = p + 64;
        const uint32_t vn = value(pn < L ? pn : L - 1);
        const uint32_t prev = lane_shr1(v, pv);
        const uint32_t nx = dpp<0x130>(v, readlane(vn, 0));  // wave_shl 1: the next element
        const bool start = p == 0 || v != prev;
        const uint64_t sm = ballot(valid && start);
        const uint64_t le = sm & (lt | (1ull << lane));
        const uint32_t o = le ? lane - (63u - (uint32_t)__builtin_clzll(le)) : po + 1 + lane;
        const uint32_t j = mod258(o);
        const bool last = p + 1 == L;
        const bool end = p + 2 == L || (p + 2 < L && nx != v);
        uint32_t cnt = last ? 1u : (uint32_t)(j <= 2) + (uint32_t)(j == 257) + (uint32_t)(end && j >= 2 && j <= 256);
        if (!valid) cnt = 0;
        const uint64_t b1 = ballot(cnt >= 1), b2 = ballot(cnt == 2);
        const uint64_t pos = q + __popcll(b1 & lt) + __popcll(b2 & lt);
        const uint32_t first = (last || j <= 2) ? v : (j == 257 ? 255u : j - 2);
        if (cnt >= 1) out[pos] = (uint8_t)first;
        if (cnt == 2) out[pos + 1] = 0;
        q += __popcll(b1) + __popcll(b2);
        po = readlane(j, 63);  // (mod 258: o itself grows along a long run)
        pv = readlane(v, 63);
        v = vn;
    }
}

// popcount of m's bits below this lane (v_mbcnt)
__device__ __forceinline__ uint32_t count_below(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// per lane: bit lane of m ? t : f (one v_cndmask on a scalar mask: no exec-mask branch)
__device__ __forceinline__ uint32_t sel(uint64_t m, uint32_t t, uint32_t f)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
// leading zeros of x, 0xFFFFFFFF for 0 (v_ffbh_u32 without the zero test)
__device__ __forceinline__ uint32_t ffbh(uint32_t x)
{
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kDrop = 0x7FFFFFF8u;  // buffer offset past every range: the store is dropped
__device__ __forceinline__ rsrc_t out_rsrc(uint8_t *p)
{
    // (readfirstlane: a pointer the compiler cannot prove uniform would get a waterfall loop)
    const uint64_t a = (uint64_t)p;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<uint8_t *>(u), (short)0, 0x7FFFFFF0, 0x00020000);
}

// emit_block for whole blocks of a tile image (L = B * B, a multiple of 64): no lane is past
// the block, so only the last step has the last-element rules; element p = 64 s + lane sits at
// LDS byte a(s) = a(0) + (s >> 1) dA + (s & 1) dB (B <= 64: dA = 2 dB, one step = 64 / B whole
// lines; B = 128: half a line), so each step's read costs one add; the previous value 0x100
// before element 0 (no byte equals it) starts its run. Branch-free: the emit rules are lane masks
// (ballots), a lane's bytes go out through a buffer store whose offset is out of range when it
// emits none. Per element with j = run offset mod 258 (transform.cpp:241-279): it emits when
// it is the block's last (a literal), j <= 2 (a literal), j = 257 (count 255) or its run ends
// (count j - 2); j = 2 at a run's end emits the literal and the count 0.
struct EmitWhole {
    uint32_t addr, dA, dB, pv, po, v, vn, q;
    rsrc_t rs;
    __device__ __forceinline__ void init(const uint8_t *D, uint32_t a0, uint32_t dA_, uint32_t dB_, uint8_t *o)
    {
        addr = a0 + dB_;
        dA = dA_;
        dB = dB_;
        pv = 0x100;  // differs from every byte: element 0 starts a run
        po = 0;
        q = 0;
        rs = out_rsrc(o);
        v = D[a0];
        vn = D[addr];
    }
    // step s (elements 64 s .. 64 s + 63); fin: the block's last step; lte_lo / lte_hi: the lanes
    // at or below this one. The elements of step s + 1 were read a step ago (readlane(vn, 0) does
    // not wait on a fresh read); those of step s + 2 are read now (past the block near its end:
    // inside the LDS image or beyond it, unused either way).
    __device__ __forceinline__ void step(const uint8_t *D, uint32_t s, bool fin, uint32_t lane, uint32_t lte_lo,
                                         uint32_t lte_hi)
    {
        addr += (s & 1) ? dB : dA - dB;
        const uint32_t vnn = D[addr];
        const uint32_t prev = lane_shr1(v, pv);
        const uint32_t nx = dpp<0x130>(v, readlane(vn, 0));  // wave_shl 1: the next element
        const uint64_t st = ballot(v != prev);
        // the run offset: from the last run start at or below this lane, else the previous step's
        const uint32_t lo = (uint32_t)st & lte_lo, hi = (uint32_t)(st >> 32) & lte_hi;
        const uint32_t t = min(ffbh(hi), ffbh(lo) + 32u);  // leading zeros of (hi, lo) when not 0
        const uint32_t o = (lo | hi) ? lane - 63u + t : po + 1u + lane;
        const uint32_t j = mod258(o);
        const uint64_t lastm = fin ? (1ull << 63) : 0ull;
        const uint64_t endm = ballot(nx != v) | (fin ? (1ull << 62) : 0ull);
        const uint64_t lit = ballot(j <= 2) | lastm;
        const uint64_t e1 = lit | endm | ballot(j == 257);
        const uint64_t e2 = ballot(j == 2) & endm & ~lastm;
        const uint32_t pos = q + count_below(e1) + count_below(e2);
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)sel(lit, v, j - 2), rs, (int)sel(e1, pos, kDrop), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)0, rs, (int)sel(e2, pos + 1, kDrop), 0, 0);
        q += (uint32_t)__builtin_popcountll(e1) + (uint32_t)__builtin_popcountll(e2);
        po = readlane(j, 63);  // (mod 258: o itself grows along a long run)
        pv = readlane(v, 63);
        v = vn;
        vn = vnn;
    }
};

// kN whole blocks of one size at once (independent chains, interleaved by the scheduler)
template <int kN>
__device__ __forceinline__ void emit_whole(const uint8_t *D, const uint32_t *a0, const uint32_t *dA,
                                           const uint32_t *dB, uint32_t L, uint8_t *const *out, uint32_t lane)
{
    const uint64_t lte = ~0ull >> (63 - lane);  // lanes at or below this one
    const uint32_t lte_lo = (uint32_t)lte, lte_hi = (uint32_t)(lte >> 32);
    EmitWhole e[kN];
#pragma unroll
    for (int k = 0; k < kN; ++k) e[k].init(D, a0[k], dA[k], dB[k], out[k]);
    for (uint32_t base = 0, s = 0; base < L; base += 64, ++s) {
        const bool fin = base + 64 == L;  // (uniform)
#pragma unroll
        for (int k = 0; k < kN; ++k) e[k].step(D, s, fin, lane, lte_lo, lte_hi);
    }
}

// emit_whole for B >= 16 (L = B * B a multiple of 256): 256 elements per step, 4 consecutive
// elements of the scan per lane (one LDS dword along a line, four bytes down a column), so the
// scans and lane reads of a step serve four elements. The run offset mod 258 (all the rules
// need) comes from a max-scan of the lanes' last run starts (biased element positions; the
// previous step's run enters as position -(j + 1) with j its last element's offset mod 258),
// then steps along the lane's elements; each lane emits 0..8 bytes at its exclusive prefix of
// the counts (one wave sum). Rules as EmitWhole.
struct EmitWhole4 {
    static constexpr uint32_t kBias = 512;
    // the read-ahead past a block's end stays inside the image (the last legal reads: a line's
    // dword at 128 kDS + 128, a column's 4 bytes from 125 kDS + 131)
    static constexpr uint32_t kMaxH = kTile * kDS + kTile, kMaxV = (kTile + 1) * kDS - 1 - 3 * kDS;
    uint32_t addr, dS, pv, po, q, v, vn;
    bool horiz;
    rsrc_t rs;
    __device__ __forceinline__ uint32_t load(const uint8_t *D, uint32_t a) const
    {
        if (horiz) return *reinterpret_cast<const uint32_t *>(D + (a < kMaxH ? a : kMaxH));
        a = a < kMaxV ? a : kMaxV;
        return (uint32_t)D[a] | (uint32_t)D[a + kDS] << 8 | (uint32_t)D[a + 2 * kDS] << 16 | (uint32_t)D[a + 3 * kDS] << 24;
    }
    // a0: this lane's first element of the block (element 4 lane); dS: the step's address increment
    __device__ __forceinline__ void init(const uint8_t *D, uint32_t a0, uint32_t dS_, bool h, uint8_t *o)
    {
        horiz = h;
        addr = a0 + dS_;
        dS = dS_;
        pv = 0x100;  // differs from every byte: element 0 starts a run
        po = 0;
        q = 0;
        rs = out_rsrc(o);
        v = load(D, a0);
        vn = load(D, addr);
    }
    __device__ __forceinline__ void step(const uint8_t *D, bool fin, uint32_t lane)
    {
        addr += dS;
        const uint32_t vnn = load(D, addr);  // two steps ahead
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) x[k] = (v >> (8 * k)) & 255u;
        const uint32_t p0 = lane_shr1(x[3], pv);
        bool S[4];
        S[0] = x[0] != p0;
#pragma unroll
        for (uint32_t k = 1; k < 4; ++k) S[k] = x[k] != x[k - 1];
        // the last run start at or below each lane (biased element position of the step)
        const uint32_t lastk = S[3] ? 3u : S[2] ? 2u : S[1] ? 1u : 0u;
        const uint32_t A = (S[0] | S[1] | S[2] | S[3]) ? 4 * lane + lastk + kBias : 0u;
        const uint32_t M = wave_scan(A, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
        uint32_t Mx = lane_shr1(M, 0u);
        const uint32_t Cb = kBias - (po + 1);  // the previous step's run
        Mx = Mx > Cb ? Mx : Cb;
        uint32_t j[4];
        j[0] = S[0] ? 0u : mod258(4 * lane + kBias - Mx);  // in 1 .. 510
#pragma unroll
        for (uint32_t k = 1; k < 4; ++k) j[k] = S[k] ? 0u : (j[k - 1] == 257u ? 0u : j[k - 1] + 1);
        // run ends: the next element differs (lane 63's next is the next step's first)
        const uint32_t nx0 = dpp<0x130>(x[0], readlane(vn, 0) & 255u);  // wave_shl 1
        const bool f63 = fin && lane == 63;
        bool end[4];
        end[0] = S[1];
        end[1] = S[2];
        end[2] = S[3] || f63;  // before the block's last element
        end[3] = nx0 != x[3];
        uint32_t cnt = 0, e1[4], e2[4], first[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const bool last = k == 3 && f63;
            const bool lit = j[k] <= 2 || last;
            e1[k] = (lit || end[k] || j[k] == 257u) ? 1u : 0u;
            e2[k] = (j[k] == 2u && end[k] && !last) ? 1u : 0u;
            first[k] = lit ? x[k] : j[k] - 2;
            cnt += e1[k] + e2[k];
        }
        const uint32_t incl = wave_sum_incl(cnt);
        uint32_t off = q + incl - cnt;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)first[k], rs, (int)(e1[k] ? off : kDrop), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)0, rs, (int)(e2[k] ? off + 1 : kDrop), 0, 0);
            off += e1[k] + e2[k];
        }
        q += readlane(incl, 63);
        po = readlane(j[3], 63);
        pv = readlane(x[3], 63);
        v = vn;
        vn = vnn;
    }
};

template <int kN>
__device__ __forceinline__ void emit_whole4(const uint8_t *D, const uint32_t *a0, const uint32_t *dS, const bool *horiz,
                                            uint32_t L, uint8_t *const *out, uint32_t lane)
{
    EmitWhole4 e[kN];
#pragma unroll
    for (int k = 0; k < kN; ++k) e[k].init(D, a0[k], dS[k], horiz[k], out[k]);
    for (uint32_t base = 0; base < L; base += 256) {
        const bool fin = base + 256 == L;  // (uniform)
#pragma unroll
        for (int k = 0; k < kN; ++k) e[k].step(D, fin, lane);
    }
}

// blocks of B <= 128: one workgroup per tile loads it once into LDS (as tile_cost_kernel
// does), then each wave emits blocks of the tile from LDS
#ifndef HC_EMIT_WPE
#define HC_EMIT_WPE 6
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HC_EMIT_WPE))) void emit_tile_kernel(EncArgs a, Ws ws)
{
    __shared__ uint8_t D[(kTile + 1) * kDS];
    __shared__ uint32_t edge[4 * kLU];  // tile_put
    const uint32_t tid = threadIdx.x;  // (lane and wave: per tile, tid_here)
    const uint64_t ntiles = ws.ctr[0];
    const bool diff = a.diff != 0;
    // the next tile's raw dwords are in flight while this one is emitted (tile_fetch / tile_put,
    // as in tile_cost_kernel): without the overlap the loads alone took half the kernel's time
    uint32_t v[kLU];
    TileAt nx;
    auto wanted = [&](const TileAt &g) __attribute__((always_inline)) { return g.ok && ws.meta[g.i].B <= kTile; };
    if (blockIdx.x < ntiles) {
        nx = tile_at(a, ws, xcd_tile(blockIdx.x, gridDim.x, ntiles));
        if (wanted(nx)) tile_fetch(nx, v, tid);
    }
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tid = tid_here(), lane = tid & 63, wv = tid >> 6;
        const TileAt g = nx;
        const bool want = wanted(g);
        HC_TC_BEGIN();
#ifdef HC_TC_PROF
        if (want) tile_put(D, edge, g, v, diff, tid, [&](uint32_t k) { HC_TC_MARK(k + 9); });
#else
        if (want) tile_put(D, edge, g, v, diff, tid);  // (its first barrier ends the previous tile)
#endif
        if (t + gridDim.x < ntiles) {
            nx = tile_at(a, ws, xcd_tile(t + gridDim.x, gridDim.x, ntiles));
            if (wanted(nx)) tile_fetch(nx, v, tid);
        }
        if (!want) continue;  // (uniform over the workgroup)
        const uint32_t i = g.i;
        const AMeta &M = ws.meta[i];
        const uint64_t W = g.W, B = M.B, tx0 = g.tx0, ty0 = g.ty0;
        const uint32_t tw = g.tw, th = g.th;
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        const uint64_t *offw = at<uint64_t>(ws, M.offs);
        const uint32_t b32 = (uint32_t)B;
        const uint32_t nbx = (tw + b32 - 1) / b32, nby = (th + b32 - 1) / b32;
        const uint64_t per_row = cdiv(W, B);
        // the wave's blocks b = wv + 4 m: each lane fetches one block's offset and scan order
        // (64 blocks per fetch), so no block waits on a global load of its own
        const uint32_t nblk = nbx * nby;
        uint64_t lane_off = 0;
        uint32_t lane_h = 0;
        // element `lane` of a whole block: line hi, offset lo; the address steps (emit_whole)
        const uint32_t lg = (uint32_t)__builtin_ctz(b32);
        const uint32_t lo = lane & (b32 - 1), hi = lane >> lg;
        auto whole_at = [&](uint32_t b, bool horiz, uint32_t &a0, uint32_t &dA, uint32_t &dB) __attribute__((always_inline)) {
            const uint32_t x0 = (b % nbx) * b32, y0 = (b / nbx) * b32;
            a0 = horiz ? (y0 + 1 + hi) * kDS + x0 + 4 + lo : (y0 + 1 + lo) * kDS + x0 + 4 + hi;
            if (b32 <= 64) {
                dB = horiz ? (64u >> lg) * kDS : 64u >> lg;
                dA = 2 * dB;
            } else {
                dA = horiz ? kDS : 1u;
                dB = horiz ? 64u : 64u * kDS;
            }
        };
        auto fetch = [&](uint32_t b, uint32_t m) __attribute__((always_inline)) {
            if (m == 0) {
                const uint32_t bl = b + 4 * lane;
                if (bl < nblk) {
                    const uint64_t kl = (ty0 / B + bl / nbx) * per_row + tx0 / B + bl % nbx;
                    lane_off = offw[kl];
                    lane_h = (sym[24 + kl / 8] >> (7 - kl % 8)) & 1;
                }
            }
        };
        auto out_of = [&](uint32_t m) __attribute__((always_inline)) {
            const uint64_t off = readlane((uint32_t)lane_off, m) | (uint64_t)readlane((uint32_t)(lane_off >> 32), m) << 32;
            return at<uint8_t>(ws, M.sym) + M.hdr + off;
        };
        if (tw % b32 == 0 && th % b32 == 0) {
            // every block whole: two blocks of the wave at a time (b, b + 4: fetch entries m, m + 1,
            // inside one 64-block fetch since m steps by 2; four at a time measured slower: SGPRs)
            auto group = [&](auto nn, uint32_t b, uint32_t m) __attribute__((always_inline)) {
                constexpr int kN = decltype(nn)::value;
                uint8_t *out[kN];
#pragma unroll
                for (int k = 0; k < kN; ++k) out[k] = out_of(m + k);
                if (b32 >= 16) {  // (uniform) 4 elements per lane: element 4 lane's address, per step +dS
                    uint32_t a0[kN], dS[kN];
                    bool hz[kN];
                    const uint32_t p = 4 * lane, ln = p >> lg, of = p & (b32 - 1);
#pragma unroll
                    for (int k = 0; k < kN; ++k) {
                        const uint32_t bb = b + 4 * k, x0 = (bb % nbx) * b32, y0 = (bb / nbx) * b32;
                        hz[k] = readlane(lane_h, m + k) != 0;
                        a0[k] = hz[k] ? (y0 + 1 + ln) * kDS + x0 + 4 + of : (y0 + 1 + of) * kDS + x0 + 4 + ln;
                        dS[k] = hz[k] ? (256u >> lg) * kDS : 256u >> lg;
                    }
                    emit_whole4<kN>(D, a0, dS, hz, b32 * b32, out, lane);
                } else {
                    uint32_t a0[kN], dA[kN], dB[kN];
#pragma unroll
                    for (int k = 0; k < kN; ++k) whole_at(b + 4 * k, readlane(lane_h, m + k) != 0, a0[k], dA[k], dB[k]);
                    emit_whole<kN>(D, a0, dA, dB, b32 * b32, out, lane);
                }
            };
            for (uint32_t b = wv; b < nblk;) {
                const uint32_t m = ((b - wv) >> 2) & 63;
                fetch(b, m);
                if (b + 4 < nblk) {
                    group(std::integral_constant<int, 2>{}, b, m);
                    b += 8;
                } else {
                    group(std::integral_constant<int, 1>{}, b, m);
                    b += 4;
                }
            }
        } else {
            for (uint32_t b = wv; b < nblk; b += 4) {
                const uint32_t m = ((b - wv) >> 2) & 63;
                fetch(b, m);
                const uint32_t bx = b % nbx, by = b / nbx;
                const uint32_t x0 = bx * b32, y0 = by * b32;
                const uint32_t sx = tw - x0 < b32 ? tw - x0 : b32, sy = th - y0 < b32 ? th - y0 : b32;
                const bool horiz = readlane(lane_h, m) != 0;
                uint8_t *out = out_of(m);
                if (sx == b32 && sy == b32) {  // (uniform) a whole block
                    uint32_t a0, dA, dB;
                    whole_at(b, horiz, a0, dA, dB);
                    emit_whole<1>(D, &a0, &dA, &dB, b32 * b32, &out, lane);
                } else {
                    const uint32_t inner = horiz ? sx : sy;
                    const float inv = 1.0f / (float)inner;
                    auto value = [&](uint32_t p) -> uint32_t {
                        const uint32_t a1 = div_small(p, inner, inv), b1 = p - a1 * inner;
                        const uint32_t xl = x0 + (horiz ? b1 : a1), yl = y0 + (horiz ? a1 : b1);
                        return DT(yl + 1, xl);
                    };
                    emit_block(value, sx * sy, out, lane);
                }
            }
        }
        HC_TC_MARK(12);
    }
}

// blocks of B >= 256 (few per matrix): one wave per block straight from memory
__global__ __launch_bounds__(256) void emit_big_kernel(EncArgs a, Ws ws)
{
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t items = ws.ctr[1];
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < items; t += (uint64_t)gridDim.x * 4) {
        const uint32_t i = find_item(ws.idx[1], a.n, t, ws.ctr[8 + 1]);
        const AMeta &M = ws.meta[i];
        if (M.status || M.B <= kTile) continue;
        uint64_t k = t - ws.idx[1][i];
        uint32_t c = kTileCand;
        while (c < kCand - 1 && k >= M.nbc[c]) k -= M.nbc[c++];
        if (c != M.best) continue;
        const uint64_t W = M.w, H = M.h, B = M.B;
        const uint64_t per_row = cdiv(W, B);
        const uint64_t x0 = (k % per_row) * B, y0 = (k / per_row) * B;
        const uint32_t sx = (uint32_t)(W - x0 < B ? W - x0 : B), sy = (uint32_t)(H - y0 < B ? H - y0 : B);
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        const bool horiz = (sym[24 + k / 8] >> (7 - k % 8)) & 1;
        const uint8_t *mat = a.in + a.in_offs[i];
        const bool diff = a.diff != 0;
        const uint32_t inner = horiz ? sx : sy;
        const float inv = 1.0f / (float)inner;
        auto value = [&](uint32_t p) -> uint32_t {
            const uint32_t a1 = div_small(p, inner, inv), b1 = p - a1 * inner;
            const uint64_t x = x0 + (horiz ? b1 : a1), y = y0 + (horiz ? a1 : b1);
            const uint64_t lin = y * W + x;
            uint32_t v = mat[lin];
            if (diff) v = (v - (lin ? mat[lin - 1] : 0u)) & 0xFFu;
            return v;
        };
        emit_block(value, sx * sy, at<uint8_t>(ws, M.sym) + M.hdr + at<uint64_t>(ws, M.offs)[k], lane);
    }
}

// adaptive failures (4 / 6 / 12 / capacity) replace whatever the FGK stage reported
__global__ void status_fix_kernel(Ws ws, uint32_t n, int32_t *status, uint64_t *out_lens)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && ws.meta[i].status) {
        status[i] = ws.meta[i].status;
        out_lens[i] = 0;
    }
}

// --------------------------------------------------------------------------- decode ------

struct DecArgs {
    const uint8_t *in;
    const uint64_t *in_offs, *in_lens;
    uint32_t n;
    uint8_t *out;
    const uint64_t *out_offs, *out_caps;
    uint64_t *out_lens;
    int32_t *status;
};

constexpr uint32_t kSub = 2048;        // symbols per sub-chunk
constexpr uint32_t kSubPerChunk = 8;   // sub-chunks per walked chunk (16384 symbols)
#ifndef HC_ZCAP
#define HC_ZCAP 1024
#endif
constexpr uint32_t kZcap = HC_ZCAP;     // Z entries a sub-chunk keeps (more: every symbol is tested; 512: C4m 5.6 ms, 1024: 3.0)
constexpr uint32_t kWinLook = 64;      // par_z: a reset machine must rejoin s0 within this
constexpr uint32_t kWinCap = 4096;     // par_scan: a longer window falls back to the serial pass
constexpr uint64_t kParMin = 1ull << 20;  // block symbols from which a stream takes this pass
#ifdef HC_DEBUG_HOOKS
// debug build: hc_debug_set_par_min lowers the threshold so that tests run the pass on small
// streams (all of the serial pass's edge cases through the parallel one)
__device__ uint64_t g_par_min = kParMin;
static uint64_t g_par_min_host = kParMin;  // its host copy (adapt_decode_work_bound)
__device__ __forceinline__ uint64_t par_min() { return g_par_min; }
// hc_debug_set_par_skew: par_walk enters every odd chunk this many output bytes off its predicted
// entry (mod W H), so tests exercise par_fix's re-runs and its repair of the starts[] entries a
// wrong walk wrote
__device__ uint64_t g_par_skew = 0;
#else
__device__ __forceinline__ uint64_t par_min() { return kParMin; }
#endif
constexpr uint32_t kDense = 0xFFFFFFFFu;

struct PSub {
    uint32_t F;   // composed transition function of the sub-chunk's symbols
    uint32_t s0;  // no-reset state before its first symbol
    uint32_t L;   // no-reset output bytes of its symbols
    uint32_t zn;  // Z entries (kDense: too many, all symbols are tested)
    uint64_t o0;  // no-reset output offset at its first symbol (par_scan)
};
struct PChk {
    uint64_t q0, o_in;  // par_scan: the walk starts at symbol q0 <= the chunk start, offset o_in,
    uint32_t r_in;      // state r_in
    uint32_t st;        // par_walk: status
    uint64_t o_q;       // the process at the chunk start (offset, state; r_q 0xFF: not reached)
    uint32_t r_q, r_out;
    uint64_t o_out;     // ... and at its end
    uint64_t e_lo, e_hi;  // par_walk: the lowest and highest start entries it wrote (e_lo > e_hi:
                          // none); a walk from a wrong entry numbers its blocks wrongly, and par_fix
                          // rewrites every entry in such a range from the exact process
};

// parallel block-boundary pass (bounds_par below): the data a stream of `cap` symbols reserves
// for it in its slab (none below kParMin symbols)
__device__ inline uint64_t par_subs(uint64_t cap) { return cap >= par_min() ? cdiv(cap, kSub) : 0; }
__device__ inline uint64_t par_bytes(uint64_t cap)
{
    const uint64_t ns = par_subs(cap);
    return align_up(sizeof(PSub) * ns, 16) + align_up(sizeof(PChk) * cdiv(ns, kSubPerChunk), 16) +
           2 * align_up(4ull * kZcap * ns, 16) + align_up(kSub / 4 * ns, 16);
}

// u64 block-start entries per stream (W H <= cap, W, H >= 8). Mode 0 records every block:
// ceil(W/B) ceil(H/B) <= (W + 7)(H + 7) / 64 for B >= 8, and (W + 7)(H + 7) / 64 <= WH / 32 + 16
// <=> 7W + 7H + 49 <= WH + 1024 <=> 0 <= (W - 7)(H - 7) + 975, true for W, H >= 8; mode 1 far
// fewer; mode 2 <= 4 W H / 1024 + 1; forged headers that would need more take larger groups
// (dec_header_kernel)
__device__ __forceinline__ uint64_t group_entries_bound(uint64_t cap) { return cap / 32 + 16; }

// symbols the FGK stage may write: the count, unless the payload cannot hold it (the first symbol
// takes >= 8 bits, every later one >= 1), which the FGK decoder reports as 9 without writing
__device__ __forceinline__ uint64_t sym_cap(uint64_t count, uint64_t len)
{
    const uint64_t avail = (len - 9) * 8;
    return count > (avail >= 8 ? avail - 7 : 0) ? 0 : count;
}

// headers of the outer stream (main.cpp:90-104): symbol capacity per stream
__global__ __launch_bounds__(1024) void dec_plan_kernel(DecArgs a, Ws ws)
{
    auto need = [&](uint32_t i, uint64_t *v) {
        const uint64_t len = a.in_lens[i];
        const uint8_t *p = a.in + a.in_offs[i];
        uint64_t count = 0;
        if (len >= 9)
            for (int b = 7; b >= 0; --b) count = count << 8 | p[b];
        const bool ok = len >= 9 && (p[8] & HC_FLAG_ADAPT);
        const uint64_t oc = a.out_caps[i];
        const uint64_t cap = sym_cap(count, len);
        v[0] = ok ? align_up(cap + 64, 16) + align_up(8 * group_entries_bound(oc) + oc / kChunk + 16, 16) + par_bytes(cap)
                  : 0;
    };
    auto put = [&](uint32_t i, const uint64_t *base) {
        uint64_t v[1];
        need(i, v);
        AMeta &m = ws.meta[i];
        const uint64_t len = a.in_lens[i];
        const uint8_t *p = a.in + a.in_offs[i];
        m.status = len < 9 ? HC_ERR_HEADER : ((p[8] & HC_FLAG_ADAPT) ? 0 : HC_ERR_UNSUPPORTED);
        m.diff = len >= 9 ? (p[8] & HC_FLAG_DIFF) != 0 : 0;
        m.slab = ws.slab0 + base[0];
        if (m.status == 0 && m.slab + v[0] > ws.slab_end) m.status = HC_ERR_CAPACITY;
        m.sym = m.slab;
        uint64_t count = 0;
        if (len >= 9)
            for (int b = 7; b >= 0; --b) count = count << 8 | p[b];
        const uint64_t cap = m.status ? 0 : sym_cap(count, len);
        m.starts = m.slab + align_up(cap + 64, 16);
        m.csum = m.starts + 8 * group_entries_bound(a.out_caps[i]);
        // the parallel boundary pass's data after the chunk sums: sub-chunk records, chunk
        // records, Z entries, packed s0 (par_bytes)
        const uint64_t nsub = par_subs(cap);
        m.pcap = nsub != 0;
        m.par = 0;
        m.psub = align_up(m.csum + a.out_caps[i] / kChunk + 16, 16);
        m.pchk = m.psub + align_up(sizeof(PSub) * nsub, 16);
        m.pz = m.pchk + align_up(sizeof(PChk) * cdiv(nsub, kSubPerChunk), 16);
        m.pzi = m.pz + align_up(4ull * kZcap * nsub, 16);
        m.ps0 = m.pzi + align_up(4ull * kZcap * nsub, 16);
        ws.sym_offs[i] = m.sym;
        ws.sym_caps[i] = cap;
        ws.sym_lens[i] = 0;
        ws.lens2[i] = m.status ? 0 : len;
    };
    __shared__ uint64_t tot[1];
    wg_scan<1>(a.n, need, put, tot);
}

// headers.cpp:65-105 on the decoded symbols, then the unblock groups and undiff chunks
__global__ __launch_bounds__(1024) void dec_header_kernel(DecArgs a, Ws ws)
{
    auto parse = [&](uint32_t i) {
        AMeta &m = ws.meta[i];
        m.nb = m.groups = m.chunks = 0;
        if (m.status == 0 && a.status[i] != 0) m.status = a.status[i];  // the FGK stage's (8 / 9 / ...)
        if (m.status) return;
        const uint64_t count = ws.sym_lens[i];
        const uint8_t *s = at<uint8_t>(ws, m.sym);
        m.count = count;
        if (count < 24) {  // headers.cpp:67-71
            m.status = HC_ERR_ADAPT_HEADER;
            return;
        }
        uint64_t f[3] = {0, 0, 0};
        for (int k = 0; k < 3; ++k)
            for (int b = 0; b < 8; ++b) f[k] = f[k] << 8 | s[8 * k + b];
        const uint64_t w = f[0], h = f[1], b = f[2];
        if (b == 0) {  // transform.cpp:415 divides by it (the reference dies by SIGFPE)
            m.status = HC_ERR_BLOCK_SIZE;
            return;
        }
        const uint64_t nb = nblocks(w, h, b);
        if (count - 24 < cdiv(nb, 8)) {  // headers.cpp:94-98
            m.status = HC_ERR_ADAPT_DIRS;
            return;
        }
        if (w != 0 && h > (1ull << 36) / w) {  // the reference: bad_alloc
            m.status = HC_ERR_TOO_LARGE;
            return;
        }
        m.w = w;
        m.h = h;
        m.B = b;
        m.nb = nb;
        m.hdr = 24 + cdiv(nb, 8);
        if (w * h > a.out_caps[i]) {
            m.status = HC_ERR_CAPACITY;
            a.out_lens[i] = w * h;
            return;
        }
        const bool pow2 = (b & (b - 1)) == 0;
        m.tiles = 0;
        if (pow2 && b >= 8 && b <= kTile) {  // tiles; every block's start is recorded
            m.mode = 0;
            m.K = 1;
            m.groups = 0;
            m.tiles = cdiv(w, kTile) * cdiv(h, kTile);
        } else if (pow2 && b > kTile) {
            m.mode = 1;
            m.K = 1;
            m.groups = nb;
        } else {  // any other block size (a forged header): groups of >= 1024 bytes
            const uint64_t bx = b < w ? b : w, by = b < h ? b : h;
            const uint64_t area = bx * by;
            m.mode = 2;
            m.K = area >= kGroupBytes ? 1 : cdiv(kGroupBytes, area ? area : 1);
            m.groups = cdiv(nb, m.K);
        }
        // the group-start entries the bounds pass writes (mode 0: one per block) must fit the
        // ones reserved for this stream (dec_plan: group_entries_bound of the output capacity).
        // Genuine streams always do; a forged header with a matrix 1..7 wide or high can name
        // more blocks than that, and takes K-block groups large enough to fit instead
        const uint64_t room = group_entries_bound(a.out_caps[i]);
        const uint64_t ents = m.mode == 0 ? nb : m.groups;
        if (ents > room) {
            const uint64_t bx = b < w ? b : w, by = b < h ? b : h, area = bx * by;
            uint64_t K = area >= kGroupBytes ? 1 : cdiv(kGroupBytes, area ? area : 1);
            if (cdiv(nb, K) > room) K = cdiv(nb, room);
            m.mode = 2;
            m.K = K;
            m.groups = cdiv(nb, K);
            m.tiles = 0;
        }
        m.ents = m.mode == 0 ? nb : m.groups;
        m.chunks = m.diff ? cdiv(w * h, kChunk) : 0;
        // many block symbols: the parallel boundary pass (the slab holds its data, dec_plan)
        m.par = m.pcap && nb && count > m.hdr && count - m.hdr >= par_min();
        m.nsub = m.par ? cdiv(count - m.hdr, kSub) : 0;
        m.nchk = cdiv(m.nsub, kSubPerChunk);
        m.pfall = 0;
        m.preruns = 0;
    };
    for (uint32_t i = threadIdx.x; i < a.n; i += blockDim.x) parse(i);
    __syncthreads();
    auto need = [&](uint32_t i, uint64_t *v) {
        v[0] = ws.meta[i].status ? 0 : ws.meta[i].groups;
        v[1] = ws.meta[i].status ? 0 : ws.meta[i].chunks;
        v[2] = ws.meta[i].status ? 0 : ws.meta[i].tiles;
        v[3] = ws.meta[i].status ? 0 : ws.meta[i].nsub;
    };
    auto put = [&](uint32_t i, const uint64_t *base) {
        ws.idx[0][i] = base[0];
        ws.idx[1][i] = base[1];
        ws.idx[2][i] = base[2];
        ws.idx[3][i] = base[3];
    };
    __shared__ uint64_t tot[4], uni[4];
    wg_scan<4>(a.n, need, put, tot, uni);
    if (threadIdx.x == 0) {
        for (int k = 0; k < 4; ++k) {
            ws.idx[k][a.n] = tot[k];
            ws.ctr[k] = tot[k];
            ws.ctr[8 + k] = uni[k];
        }
    }
}

// The revert machine (transform.cpp:137-159) as state r in 0..3 (equal literals seen; 3 = the
// next symbol is a count): a literal equal to the previous symbol moves r -> r + 1, another one
// r -> 1, a count 3 -> 0; from 0 both give 1, so the symbol before a block start never matters.
// Transition functions as 4 x 2-bit tables, composed by wave scans.
// A transition function is a 4-byte table (byte x = the state x goes to); g after f is one
// v_perm_b32 (the bytes of g picked by the bytes of f).
constexpr uint32_t kFsmEq = 0x00030201u;  // 0->1 1->2 2->3 3->0
constexpr uint32_t kFsmNe = 0x00010101u;  // 0->1 1->1 2->1 3->0
constexpr uint32_t kFsmId = 0x03020100u;

__device__ __forceinline__ uint32_t fsm_then(uint32_t g, uint32_t f)  // x -> g(f(x))
{
    return __builtin_amdgcn_perm(0u, g, f);
}
__device__ __forceinline__ uint32_t fsm_at(uint32_t f, uint32_t x) { return (f >> (8 * x)) & 0xFFu; }
__device__ __forceinline__ uint32_t fsm_scan(uint32_t f)
{
    return wave_scan(f, kFsmId, [](uint32_t later, uint32_t earlier) { return fsm_then(later, earlier); });
}

__device__ __forceinline__ uint32_t block_size(const AMeta &m, uint64_t k, uint64_t *x0, uint64_t *y0,
                                               uint64_t *sx, uint64_t *sy)
{
    const uint64_t per_row = cdiv(m.w, m.B);
    *x0 = (k % per_row) * m.B;
    *y0 = (k / per_row) * m.B;
    *sx = m.w - *x0 < m.B ? m.w - *x0 : m.B;
    *sy = m.h - *y0 < m.B ? m.h - *y0 : m.B;
    return 0;
}

// Block geometry of one adaptive stream (transform.cpp:25-62, 410-418): blocks in row-major
// order, block row by starting at output offset by * B * W, block bx of it at bx * B * sy (sy
// the row's height). 64-bit divisions by a double reciprocal, corrected (exact below 2^53).
__device__ __forceinline__ uint64_t udiv(uint64_t a, uint64_t d, double inv)
{
    uint64_t q = (uint64_t)((double)a * inv);
    uint64_t p = q * d;
    while (p > a) {
        --q;
        p -= d;
    }
    while (a - p >= d) {
        ++q;
        p += d;
    }
    return q;
}
struct Geo {
    uint64_t W, H, B, per_row, nbr, nb, RB, total;
    double inv_RB;
    __device__ void init(uint64_t w, uint64_t h, uint64_t b)
    {
        W = w;
        H = h;
        B = b;
        per_row = cdiv(w, b);
        nbr = cdiv(h, b);
        nb = per_row * nbr;
        RB = b * w;
        total = w * h;
        inv_RB = RB ? 1.0 / (double)RB : 0.0;
    }
    __device__ uint64_t sy(uint64_t by) const { return H - by * B < B ? H - by * B : B; }
    __device__ uint64_t sx(uint64_t bx) const { return W - bx * B < B ? W - bx * B : B; }
    // the block holding output offset o < total: (bx, by) and o - its first offset
    __device__ void locate(uint64_t o, uint64_t &bx, uint64_t &by, uint64_t &rel) const
    {
        by = udiv(o, RB, inv_RB);
        if (by >= nbr) by = nbr - 1;
        const uint64_t r = o - by * RB, area = B * sy(by);
        bx = udiv(r, area, 1.0 / (double)area);
        if (bx >= per_row) bx = per_row - 1;
        rel = r - bx * area;
    }
    // o is the first byte of a block
    __device__ bool is_start(uint64_t o) const
    {
        if (o >= total) return false;
        uint64_t bx, by, rel;
        locate(o, bx, by, rel);
        return rel == 0;
    }
};

// The serial boundary process of one stream (transform.cpp:330-361 running revertRLEBlock,
// transform.cpp:162-187, block by block), from any entry: symbols from `pos` in machine state r
// at output offset E(blk) + got. One wave, 256 symbols per step (4 per lane, from dword loads
// re-aligned by v_alignbyte, the next step's already in flight); a scan of the transition
// functions gives each symbol's state, hence its output length (count: the symbol, literal: 1);
// a scan of lengths finds the first symbol where the block's byte count is reached. A block that
// ends inside the step re-scans the rest of the same registers from state 0. The start of every
// K-th block (group) at or after `rec_from` is recorded for the unblock waves.
#ifndef HC_BOUNDS_W
#define HC_BOUNDS_W 1
#endif
constexpr uint32_t kBW = HC_BOUNDS_W;   // symbol dwords per lane and step
constexpr uint32_t kBStep = 256 * kBW;  // symbols per step
struct BWalk {
    const uint32_t *sw;  // the stream's symbols as dwords (16-aligned slab, 64 bytes of slack)
    uint64_t nsym;       // symbols (adaptive header included)
    uint64_t hdr;        // first block symbol
    uint64_t *starts;
    uint64_t K, ents;
    uint64_t W, H, B, per_row, nb;  // geometry (Geo geo() for the rest: entries and exits only)
    uint32_t lane;
    // process state
    uint64_t pos, blk, got, want;
    uint64_t bx, by, kq, gq;  // block column / row; blk mod K, blk / K (K = 1 in mode 0: every block)
    uint32_t r, last;
    uint64_t e_lo, e_hi;  // the lowest and highest entries written (e_lo > e_hi: none)

    __device__ void init(const AMeta &M, const uint8_t *sym, uint64_t *st, uint32_t l)
    {
        sw = reinterpret_cast<const uint32_t *>(sym);
        nsym = M.count;
        hdr = M.hdr;
        starts = st;
        K = M.K;
        ents = M.ents;
        W = M.w;
        H = M.h;
        B = M.B;
        per_row = cdiv(W, B);
        nb = per_row * cdiv(H, B);
        lane = l;
        e_lo = ~0ull;
        e_hi = 0;
    }
    // starts[e] := q (lane 0 stores; every lane tracks the range)
    __device__ __forceinline__ void record(uint64_t e, uint64_t q)
    {
        if (lane == 0) starts[e] = q;
        e_lo = e < e_lo ? e : e_lo;
        e_hi = e > e_hi ? e : e_hi;
    }
    __device__ Geo geo() const
    {
        Geo g;
        g.init(W, H, B);
        return g;
    }
    __device__ uint64_t block_want() const
    {
        return (W - bx * B < B ? W - bx * B : B) * (H - by * B < B ? H - by * B : B);
    }
    __device__ uint64_t entry() const { return gq; }  // when kq == 0
    // step to the next block; its group-start entry (~0 if it starts no group)
    __device__ uint64_t next_block()
    {
        if (++bx == per_row) {
            bx = 0;
            ++by;
        }
        if (++kq == K) {
            kq = 0;
            ++gq;
        }
        return kq ? ~0ull : entry();
    }
    // output offset of the process: the current block's first byte + got
    __device__ uint64_t offset() const
    {
        return blk >= nb ? W * H : by * B * W + bx * B * (H - by * B < B ? H - by * B : B) + got;
    }
    // enter at symbol q in state r0 at output offset o (a block start resets the state)
    __device__ void enter(uint64_t q, uint32_t r0, uint64_t o, uint64_t rec_from)
    {
        pos = q;
        r = r0;
        last = q > hdr ? reinterpret_cast<const uint8_t *>(sw)[q - 1] : 0u;
        got = 0;
        if (o >= W * H) {
            blk = nb;
            bx = by = kq = gq = 0;
            want = 0;
            return;
        }
        uint64_t rel;
        geo().locate(o, bx, by, rel);
        blk = by * per_row + bx;
        got = rel;
        want = block_want();
        kq = blk % K;
        gq = blk / K;
        if (got == 0) {
            r = 0;
            if (kq == 0 && q >= rec_from && entry() < ents) record(entry(), q);
        }
    }
    __device__ void load(uint64_t p, uint32_t *w) const
    {
        const uint64_t d = (p >> 2) + kBW * lane;
#pragma unroll
        for (uint32_t j = 0; j <= kBW; ++j) w[j] = 4 * (d + j) < nsym ? sw[d + j] : 0u;
    }
    // run over the symbols below q1 (<= nsym): 0 when q1 is reached with blocks left, or the
    // reference's exit there: 13 (a count overshoots its block), 14 (the stream ends inside a
    // block), 15 (symbols left after the last block); blk == nb with pos == nsym: 0 (done)
    // kWhole: the whole stream from its start (q1 = nsym, every start recorded)
    template <bool kWhole = false>
    __device__ int run(uint64_t q1, uint64_t rec_from)
    {
        if constexpr (kWhole) {
            q1 = nsym;
            rec_from = 0;
        }
        uint32_t cur[kBW + 1];
        load(pos, cur);
        while (blk < nb) {
            const uint64_t avail = q1 - pos;
            const uint32_t m = avail < kBStep ? (uint32_t)avail : kBStep;
            if (m == 0) return pos == nsym ? HC_ERR_BLOCK_EOF : 0;  // transform.cpp:170-174
            uint32_t nxt[kBW + 1];
            load(pos + kBStep, nxt);  // the next step's symbols, in flight during this one
            constexpr uint32_t kB = 4 * kBW;
            uint32_t x[kB];
#pragma unroll
            for (uint32_t j = 0; j < kBW; ++j) {
                const uint32_t w = __builtin_amdgcn_alignbyte(cur[j + 1], cur[j], (uint32_t)(pos & 3));
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) x[4 * j + k] = kB * lane + 4 * j + k < m ? (w >> (8 * k)) & 255u : 0u;
            }
            const uint32_t up = lane_shr1(x[kB - 1], last);
            uint32_t lo = 0;  // symbols below lo belong to blocks already closed
            for (;;) {
                uint32_t f[kB], F = kFsmId;
#pragma unroll
                for (uint32_t k = 0; k < kB; ++k) {
                    const uint32_t ii = kB * lane + k;
                    const uint32_t p = k ? x[k - 1] : up;
                    f[k] = (ii >= lo && ii < m) ? (x[k] == p ? kFsmEq : kFsmNe) : kFsmId;
                    F = fsm_then(f[k], F);
                }
                const uint32_t inc = fsm_scan(F);
                uint32_t s = fsm_at(lane_shr1(inc, kFsmId), r);
                uint32_t len[kB], tot = 0;
#pragma unroll
                for (uint32_t k = 0; k < kB; ++k) {
                    const uint32_t ii = kB * lane + k;
                    len[k] = (ii >= lo && ii < m) ? (s == 3 ? x[k] : 1u) : 0u;
                    tot += len[k];
                    s = fsm_at(f[k], s);
                }
                const uint32_t acc = wave_sum_incl(tot);
                const uint64_t need = want - got;  // >= 1
                const uint64_t hit = ballot((uint64_t)acc >= need);
                if (!hit) {  // the block goes on past this step
                    got += readlane(acc, 63);
                    r = fsm_at(readlane(inc, 63), r);
                    uint32_t lx = x[0];
#pragma unroll
                    for (uint32_t k = 1; k < kB; ++k) lx = ((m - 1) % kB) == k ? x[k] : lx;
                    last = readlane(lx, (m - 1) / kB);
                    pos += m;
                    break;
                }
                const uint32_t L = (uint32_t)__builtin_ctzll(hit);
                uint32_t c = acc - tot, j = 0xFFFFFFFFu, cj = 0;
#pragma unroll
                for (uint32_t k = 0; k < kB; ++k) {
                    c += len[k];
                    if (j == 0xFFFFFFFFu && (uint64_t)c >= need) {
                        j = kB * lane + k;
                        cj = c;
                    }
                }
                j = readlane(j, L);
                cj = readlane(cj, L);
                if ((uint64_t)cj != need) return HC_ERR_BLOCK_DATA;  // transform.cpp:178-182
                lo = j + 1;
                ++blk;
                const uint64_t e = next_block();
                if (blk < nb && e < ents && pos + lo >= rec_from) record(e, pos + lo);
                // the next block starts in state 0 (the previous symbol does not matter then; at a
                // chunk exit on a block end the state is not compared either: par_fix)
                r = 0;
                got = 0;
                if (blk == nb) {
                    pos += lo;
                    return pos != nsym ? HC_ERR_LEFTOVER : 0;  // transform.cpp:354-358
                }
                want = block_want();
                if (lo == m) {  // the block ends with the step: the next starts at pos + m
                    pos += m;
                    break;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j <= kBW; ++j) cur[j] = nxt[j];
        }
        return pos != nsym ? HC_ERR_LEFTOVER : 0;
    }
};

// One wave per stream (the streams the parallel pass below does not take): the serial process
// over the whole stream.
#ifndef HC_BOUNDS_WPE
#define HC_BOUNDS_WPE 6
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HC_BOUNDS_WPE))) void bounds_kernel(DecArgs a, Ws ws)
{
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t i = blockIdx.x * 4 + wv; i < a.n; i += gridDim.x * 4) {
        const uint32_t lane = tid_here() & 63;
        AMeta &M = ws.meta[i];
        if (M.status || M.par) continue;
        BWalk w;
        w.init(M, at<uint8_t>(ws, M.sym), at<uint64_t>(ws, M.starts), lane);
        // the stream's start: block 0 in state 0
        w.pos = M.hdr;
        w.r = w.last = 0;
        w.blk = w.got = w.bx = w.by = w.kq = w.gq = 0;
        w.want = w.block_want();
        if (lane == 0 && w.nb) w.starts[0] = M.hdr;
        const int status = w.run<true>(0, 0);
        if (lane == 0) M.status = status;
    }
}

// ------------------------------------------------------ parallel block-boundary pass ------
// For a stream of many symbols (C4: 11 M), the serial process above is one wave's chain of
// block ends. The parallel pass (model and argument: tests/bounds_par_model.py):
//   par_fsm    per 2048-symbol sub-chunk: the composed transition function of its symbols;
//   par_entry  per stream: a scan of those: the no-reset machine's state s0 at each sub-chunk;
//   par_z      per sub-chunk: s0, lengths and offsets of every symbol without block resets
//              (packed s0 kept), and Z: the symbols where a reset (a block start) would change
//              some length before the reset machine rejoins s0;
//   par_scan   per stream, one wave: Z in order with the running correction D: z is a block
//              start iff O0(z) + D is a block's first byte; there the true machine runs until it
//              rejoins s0 (new D). Writes each 16384-symbol chunk's predicted entry;
//   par_walk   per chunk: the serial process from its predicted entry: block starts, error,
//              exit;
//   par_fix    per stream: entries checked against the previous chunk's exit in order, chunks
//              that differ re-run from the exact exit (so the result is exact whatever par_scan
//              predicted); the first error is the stream's status.
__device__ __forceinline__ uint32_t fsm_step(uint32_t x, uint32_t xp) { return x == xp ? kFsmEq : kFsmNe; }

// symbols p0 + 32 lane .. + 31 (< end) as 8 dwords per lane (bytes past end: 0); returns the
// symbol before the lane's first (lane 0: before p0, 0 at the block data start)
__device__ __forceinline__ uint32_t load_sub(const uint8_t *sym, uint64_t hdr, uint64_t p0, uint64_t end, uint32_t lane,
                                             uint32_t *w)
{
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(sym);
    const uint64_t b = p0 + 32 * lane;
    const uint64_t d = b >> 2;
    uint32_t raw[9];
#pragma unroll
    for (uint32_t j = 0; j < 9; ++j) raw[j] = 4 * (d + j) < end + 4 ? sw[d + j] : 0u;  // (slab slack)
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        uint32_t v = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], (uint32_t)(b & 3));
        const uint64_t q = b + 4 * j;  // mask bytes at or past end
        if (q + 4 > end) v = q >= end ? 0u : (v & (0xFFFFFFFFu >> (8 * (uint32_t)(q + 4 - end))));
        w[j] = v;
    }
    const uint32_t prev_lane = lane_shr1(w[7] >> 24, 0u);
    const uint32_t before = p0 > hdr ? (uint32_t)sym[p0 - 1] : 0u;
    return lane == 0 ? before : prev_lane;
}
// the lane's 32 symbols' composed transition function (symbols at or past end: identity)
__device__ __forceinline__ uint32_t lane_fsm(const uint32_t *w, uint32_t prev, uint64_t p, uint64_t end)
{
    uint32_t F = kFsmId, xp = prev;
#pragma unroll
    for (uint32_t t = 0; t < 32; ++t) {
        const uint32_t x = (w[t >> 2] >> (8 * (t & 3))) & 255u;
        F = p + t < end ? fsm_then(fsm_step(x, xp), F) : F;
        xp = x;
    }
    return F;
}

// per-stream data of the pass, in the stream's slab
__device__ __forceinline__ PSub *psub(const Ws &ws, const AMeta &M) { return at<PSub>(ws, M.psub); }
__device__ __forceinline__ PChk *pchk(const Ws &ws, const AMeta &M) { return at<PChk>(ws, M.pchk); }

// the sub-chunk of work item t: stream i, sub j
__device__ __forceinline__ bool sub_item(const DecArgs &a, const Ws &ws, uint64_t t, uint32_t &i, uint64_t &j)
{
    i = find_item(ws.idx[3], a.n, t, ws.ctr[8 + 3]);
    const AMeta &M = ws.meta[i];
    j = t - ws.idx[3][i];
    return M.status == 0 && M.par && j < M.nsub;
}

__global__ __launch_bounds__(256) void par_fsm_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t items = ws.ctr[3];
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < items; t += (uint64_t)gridDim.x * 4) {
        uint32_t i;
        uint64_t j;
        if (!sub_item(a, ws, t, i, j)) continue;
        const AMeta &M = ws.meta[i];
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        const uint64_t p0 = M.hdr + j * kSub, end = p0 + kSub < M.count ? p0 + kSub : M.count;
        uint32_t w[8];
        const uint32_t prev = load_sub(sym, M.hdr, p0, end, lane, w);
        const uint32_t F = fsm_scan(lane_fsm(w, prev, p0 + 32 * lane, end));
        if (lane == 63) psub(ws, M)[j].F = F;
    }
}

// one wave per stream: s0 at every sub-chunk (the machine starts in state 0 at the block data)
__global__ __launch_bounds__(64) void par_entry_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id();
    for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        const AMeta &M = ws.meta[i];
        if (M.status || !M.par) continue;
        PSub *S = psub(ws, M);
        uint32_t carry = 0;
        for (uint64_t b = 0; b < M.nsub; b += 64) {
            const bool ok = b + lane < M.nsub;
            const uint32_t f = ok ? S[b + lane].F : kFsmId;
            const uint32_t inc = fsm_scan(f);
            if (ok) S[b + lane].s0 = fsm_at(lane_shr1(inc, kFsmId), carry);
            carry = fsm_at(readlane(inc, 63), carry);
        }
    }
}

// per sub-chunk: packed s0 (2 bits per symbol), no-reset bytes L, and the Z entries
// (offset in the sub-chunk's no-reset output << 11 | symbol index in the sub-chunk)
__global__ __launch_bounds__(256) void par_z_kernel(DecArgs a, Ws ws)
{
    __shared__ uint8_t X[4][kSub + kWinLook + 4];  // symbols p0 - 4 .. end + kWinLook
    __shared__ uint8_t S0[4][kSub + kWinLook];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t items = ws.ctr[3];
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < items; t += (uint64_t)gridDim.x * 4) {
        uint32_t i;
        uint64_t j;
        if (!sub_item(a, ws, t, i, j)) continue;
        const AMeta &M = ws.meta[i];
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        PSub *SB = psub(ws, M);
        const uint64_t n = M.count;
        const uint64_t p0 = M.hdr + j * kSub, end = p0 + kSub < n ? p0 + kSub : n;
        const uint32_t cnt = (uint32_t)(end - p0);
        uint32_t w[8];
        const uint32_t prev = load_sub(sym, M.hdr, p0, end, lane, w);
        const uint32_t Fl = lane_fsm(w, prev, p0 + 32 * lane, end);
        const uint32_t inc = fsm_scan(Fl);
        uint32_t s = fsm_at(lane_shr1(inc, kFsmId), SB[j].s0);  // no-reset state at the lane's first
        uint8_t *Xw = X[wv] + 4, *Sw = S0[wv];
        // per symbol: s0 (packed and in LDS), no-reset length
        uint32_t pk0 = 0, pk1 = 0, lsum = 0, xp = prev;
#pragma unroll
        for (uint32_t k = 0; k < 32; ++k) {
            const uint32_t x = (w[k >> 2] >> (8 * (k & 3))) & 255u;
            const bool ok = 32 * lane + k < cnt;
            if (k < 16) pk0 |= s << (2 * k);
            else pk1 |= s << (2 * (k - 16));
            Xw[32 * lane + k] = (uint8_t)x;
            Sw[32 * lane + k] = (uint8_t)s;
            lsum += ok ? (s == 3 ? x : 1u) : 0u;
            s = ok ? fsm_at(fsm_step(x, xp), s) : s;
            xp = x;
        }
        if (lane == 0) Xw[-1] = (uint8_t)prev;
        uint32_t *pk = at<uint32_t>(ws, M.ps0) + j * (kSub / 16);
        pk[2 * lane] = pk0;
        pk[2 * lane + 1] = pk1;
        // lookahead: the next sub-chunk's first kWinLook symbols and their s0
        {
            const uint64_t q = end + lane;
            const uint32_t x = q < n ? sym[q] : 0u;
            const uint32_t xq = lane_shr1(x, cnt ? (uint32_t)sym[end - 1] : 0u);
            const uint32_t f = q < n ? fsm_step(x, xq) : kFsmId;
            const uint32_t sc = end < n ? SB[j + 1].s0 : 0u;
            const uint32_t li = fsm_scan(f);
            Xw[cnt + lane] = (uint8_t)x;
            Sw[cnt + lane] = (uint8_t)fsm_at(lane_shr1(li, kFsmId), sc);
        }
        const uint32_t lacc = wave_sum_incl(lsum);
        const uint32_t obase = lacc - lsum;  // no-reset output before the lane's first symbol
        if (lane == 63) SB[j].L = lacc;
        __builtin_amdgcn_wave_barrier();
        // Z: from each symbol p, the machine reset to 0 there, until it rejoins s0 (at most
        // kWinLook symbols; a window that does not rejoin counts as Z: the scanner simulates it)
        uint32_t zmask = 0;
        const uint32_t lim = cnt + kWinLook < (uint32_t)(n - p0) ? cnt + kWinLook : (uint32_t)(n - p0);
        // the machine reset to 0 at symbol p, until it rejoins s0: whether a length differs (Z),
        // and for the scanner's fast path (zinfo) the window's length, its length correction
        // and its output without the last symbol (0: no fast path)
        auto window = [&](uint32_t p, uint32_t &info) __attribute__((always_inline)) -> bool {
            uint32_t u = 0, q = p, wt = 0, lt = 0;
            int32_t dl = 0;
            bool mism = false;
            while (q < lim && u != Sw[q] && q - p < kWinLook) {
                const uint32_t x = Xw[q], s0q = Sw[q];
                lt = u == 3 ? x : 1u;
                const uint32_t l0 = s0q == 3 ? x : 1u;
                mism |= lt != l0;
                dl += (int32_t)lt - (int32_t)l0;
                wt += lt;
                u = fsm_at(fsm_step(x, Xw[(int)q - 1]), u);
                ++q;
            }
            const bool synced = q < lim ? u == Sw[q] : false;
            const uint32_t wl = q - p, wo = wt - lt;
            info = synced && wl < 64 && dl >= -4096 && dl < 4096 && wo < 8192
                       ? wl | ((uint32_t)(dl + 4096) << 6) | (wo << 19) : 0u;
            return mism || (q < lim && !synced);
        };
        for (uint32_t k = 0; k < 32; ++k) {
            const uint32_t p = 32 * lane + k;
            if (p >= cnt) break;
            uint32_t info;
            if (window(p, info)) zmask |= 1u << k;
        }
        const uint32_t zc = (uint32_t)__builtin_popcount(zmask);
        const uint32_t zacc = wave_sum_incl(zc);
        const uint32_t ztot = readlane(zacc, 63);
        if (ztot <= kZcap) {
            uint32_t *Z = at<uint32_t>(ws, M.pz) + j * kZcap;
            uint32_t *ZI = at<uint32_t>(ws, M.pzi) + j * kZcap;
            uint32_t at_ = zacc - zc;
            uint32_t oo = obase;
            for (uint32_t k = 0; k < 32; ++k) {
                const uint32_t p = 32 * lane + k;
                if (p >= cnt) break;
                if ((zmask >> k) & 1u) {
                    uint32_t info;
                    (void)window(p, info);
                    ZI[at_] = info;
                    Z[at_++] = (oo << 11) | p;
                }
                const uint32_t s0p = Sw[p], x = Xw[p];
                oo += s0p == 3 ? x : 1u;
            }
        }
        if (lane == 0) SB[j].zn = ztot <= kZcap ? ztot : kDense;
        __builtin_amdgcn_wave_barrier();
    }
}

// the no-reset state s0 of symbol p (packed by par_z)
__device__ __forceinline__ uint32_t s0_at(const uint32_t *pk, uint64_t rel)
{
    return (pk[rel >> 4] >> (2 * (rel & 15))) & 3u;
}

// One workgroup per stream: Z in order with the running correction D
// (tests/bounds_par_model.py). The serial part -- D changes at every block start found in Z --
// is one wave (the consumer); the other kProd (producers) run up to kRing sub-chunks ahead of it:
// each loads a sub-chunk's record and Z entries with their window infos into an LDS ring slot
// (a dense sub-chunk: every symbol as an entry, with its symbols and states), notes in a bitmap
// the residues mod B^2 of the entries' no-reset offsets (hashed to 1024 bits), and tests the
// entries against the D the consumer last published (a version of it), noting the first
// candidate and loading the symbols around it. The consumer takes a slot whose test used the
// current version as it is; after a block start found since, the bitmap tells in one read whether
// any entry can be one under the new D (else the slot's entries are tested again). A block start
// in Z whose window par_z could describe (not split by a block end or a chunk start) takes D +=
// its correction at once; any other is simulated symbol by symbol, its window from the slot.
constexpr uint32_t kZr = kZcap / 64;  // Z entries per lane and sub-chunk
constexpr uint32_t kRing = 10;        // ring slots (sub-chunks ahead of the consumer)
constexpr uint32_t kSpinCap = 1u << 23;  // sleeps before a wait gives up (~1 s; never expected)
constexpr uint32_t kProd = 11;        // producer waves (12 waves per workgroup: registers for the consumer's paths)
struct RSlot {
    uint32_t j;      // the sub-chunk published here (0xFFFFFFFF: none yet)
    uint32_t ver;    // the D version its test used
    uint32_t first;  // first candidate under that version: entry index (dense: symbol index), ~0 none
    uint32_t zn;     // entries (kDense: dense, every symbol an entry)
    uint32_t s0, L;
    uint64_t o0;
    uint64_t wz;     // the prefetched window's block start (~0: none)
    uint32_t wx[16];  // symbols wz - 1 .. wz + 62
    uint32_t ws[4];   // s0 of wz .. wz + 63: bit planes (low 64 bits, high 64 bits)
    uint32_t bm[32];  // residues (o0 + rel) mod B^2 (mod 1024) of the entries present
    uint32_t ze[kSub];          // entries: Z (zn of them) or, dense, all symbols (offset << 11 | index)
    uint32_t zi[kZcap];         // window infos (Z entries)
    uint32_t sx[kSub / 4];      // dense: the symbols (p0 .. p0 + cnt)
    uint32_t sp[kSub / 16];     // dense: packed s0
};
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }

__global__ __launch_bounds__(64 * (kProd + 1)) void par_scan_kernel(DecArgs a, Ws ws)
{
    __shared__ RSlot ring[kRing];
    __shared__ int64_t vD[64];                // D of version v at [v % 64]
    __shared__ uint64_t vres[64];             // resume of version v
    __shared__ uint32_t sh_ver, sh_done, sh_quit;
    __shared__ uint32_t part[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        AMeta &M = ws.meta[i];
        if (M.status || !M.par) continue;  // (uniform over the workgroup)
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        const uint32_t *pk = at<uint32_t>(ws, M.ps0);
        PSub *SB = psub(ws, M);
        PChk *C = pchk(ws, M);
        const uint32_t *Zall = at<uint32_t>(ws, M.pz), *ZIall = at<uint32_t>(ws, M.pzi);
        Geo g;
        g.init(M.w, M.h, M.B);
        const uint64_t n = M.count, hdr = M.hdr, nsub = M.nsub;
        const uint64_t span = (uint64_t)kSub * kSubPerChunk;
        // fast test: below full_end every block start is a multiple of B^2 (mask = B^2 - 1) and
        // every block holds B^2 bytes
        const bool pow2 = (g.B & (g.B - 1)) == 0 && g.W % g.B == 0 && g.B <= 4096;
        const uint64_t mask = pow2 ? g.B * g.B - 1 : 0, full_end = pow2 ? (g.nbr - 1) * g.RB : 0;
        // 1. the no-reset offset of every sub-chunk (exclusive scan of L, the whole workgroup)
        {
            uint64_t carry = 0;
            constexpr uint32_t kT = 64 * (kProd + 1);
            for (uint64_t b = 0; b < nsub; b += kT) {
                const uint64_t j = b + tid;
                const uint32_t l = j < nsub ? SB[j].L : 0u;
                const uint32_t inc = wave_sum_incl(l);
                if (lane == 63) part[wv] = inc;
                __syncthreads();
                uint64_t before = carry, tot = 0;
                for (uint32_t w = 0; w < kProd + 1; ++w) {
                    before += w < wv ? part[w] : 0u;
                    tot += part[w];
                }
                if (j < nsub) SB[j].o0 = before + inc - l;
                carry += tot;
                __syncthreads();
            }
        }
        if (tid < kRing) ring[tid].j = 0xFFFFFFFFu;
        if (tid == 0) {
            sh_ver = 0;
            sh_done = 0;
            sh_quit = 0;
            vD[0] = 0;
            vres[0] = 0;
        }
        __syncthreads();  // (also makes the o0 stores visible to the workgroup)
        // the block-start test of entry e (rel << 11 | symbol index) of a sub-chunk at p0 with
        // no-reset offset o0, under (D, resume)
        auto test = [&](uint32_t e, bool ok, uint64_t p0, uint64_t o0, int64_t D, uint64_t resume)
            __attribute__((always_inline)) -> bool {
            const uint64_t base = o0 + D;
            const uint32_t rres = resume <= p0 ? 0u : (resume - p0 >= kSub ? kSub : (uint32_t)(resume - p0));
            const uint32_t bm = (uint32_t)(base & mask);
            const uint32_t rlim =
                base >= full_end ? 0u : (full_end - base > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(full_end - base));
            const uint32_t pr = e & 2047u, rel = e >> 11;
            bool hit;
            if (rel < rlim) hit = ((bm + rel) & (uint32_t)mask) == 0;
            else hit = ok && g.is_start(base + rel);
            return ok && pr >= rres && hit;
        };
        if (wv > 0) {
            // ------------------------------------------------------------- producers
            for (uint64_t j = wv - 1; j < nsub; j += kProd) {
                RSlot &R = ring[j % kRing];
                // the slot is free once the consumer is done with sub-chunk j - kRing (bounded: a
                // wait past ~1 s gives up, and the serial pass in par_fix takes over)
                for (uint32_t spin = 0; lds_ld(&sh_done) + kRing <= j && !lds_ld(&sh_quit); ++spin) {
                    if (spin > kSpinCap) {
                        lds_st(&sh_quit, 2u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (lds_ld(&sh_quit)) break;
                const PSub rec = SB[j];
                const uint64_t p0 = hdr + j * kSub;
                const uint32_t cnt = (uint32_t)((p0 + kSub < n ? p0 + kSub : n) - p0);
                const bool dense = rec.zn == kDense;
                const uint32_t items = dense ? cnt : rec.zn;
                if (lane < 32) R.bm[lane] = pow2 ? 0u : 0xFFFFFFFFu;
                __builtin_amdgcn_wave_barrier();
                if (!dense) {
                    uint32_t e[kZr], zi[kZr];
#pragma unroll
                    for (uint32_t r = 0; r < kZr; ++r) {
                        const uint32_t it = 64 * r + lane;
                        e[r] = it < items ? Zall[j * kZcap + it] : 0xFFFFFFFFu;
                        zi[r] = it < items ? ZIall[j * kZcap + it] : 0u;
                    }
#pragma unroll
                    for (uint32_t r = 0; r < kZr; ++r) {
                        R.ze[64 * r + lane] = e[r];
                        R.zi[64 * r + lane] = zi[r];
                        if (pow2 && e[r] != 0xFFFFFFFFu) {
                            const uint32_t res = (uint32_t)((rec.o0 + (e[r] >> 11)) & mask) & 1023u;
                            __hip_atomic_fetch_or(&R.bm[res >> 5], 1u << (res & 31), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                    }
                } else {  // every symbol: its no-reset offset from s0 and lengths
                    uint32_t w[8];
                    (void)load_sub(sym, hdr, p0, p0 + cnt, lane, w);
                    const uint32_t s0lo = pk[j * (kSub / 16) + 2 * lane], s0hi = pk[j * (kSub / 16) + 2 * lane + 1];
                    auto len = [&](uint32_t q) __attribute__((always_inline)) {
                        const uint32_t x = (w[q >> 2] >> (8 * (q & 3))) & 255u;
                        const uint32_t s0 = ((q < 16 ? s0lo : s0hi) >> (2 * (q & 15))) & 3u;
                        return 32 * lane + q < cnt ? (s0 == 3 ? x : 1u) : 0u;
                    };
                    uint32_t tot = 0;
#pragma unroll
                    for (uint32_t q = 0; q < 32; ++q) tot += len(q);
                    const uint32_t inc = wave_sum_incl(tot);
                    uint32_t acc = inc - tot;
#pragma unroll
                    for (uint32_t q = 0; q < 32; ++q) {
                        const uint32_t idx = 32 * lane + q;
                        R.ze[idx] = idx < cnt ? (acc << 11) | idx : 0xFFFFFFFFu;
                        if (pow2 && idx < cnt) {
                            const uint32_t res = (uint32_t)((rec.o0 + acc) & mask) & 1023u;
                            __hip_atomic_fetch_or(&R.bm[res >> 5], 1u << (res & 31), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                        acc += len(q);
                    }
#pragma unroll
                    for (uint32_t k = 0; k < 8; ++k) R.sx[8 * lane + k] = w[k];
                    R.sp[2 * lane] = s0lo;
                    R.sp[2 * lane + 1] = s0hi;
                }
                __builtin_amdgcn_wave_barrier();
                // the consumer's current version of (D, resume), and the first candidate under it
                const uint32_t v = lds_ld(&sh_ver);
                const int64_t D = vD[v % 64];
                const uint64_t resume = vres[v % 64];
                uint32_t first = 0xFFFFFFFFu;
                for (uint32_t b = 0; b < items && first == 0xFFFFFFFFu; b += 64) {
                    const uint32_t e = b + lane < items ? R.ze[b + lane] : 0xFFFFFFFFu;
                    const uint64_t m = ballot(test(e, e != 0xFFFFFFFFu, p0, rec.o0, D, resume));
                    if (m) first = b + (uint32_t)__builtin_ctzll(m);
                }
                // the window around it (a Z entry's; a dense sub-chunk has its symbols in the slot):
                // symbols z - 1 .. z + 62, s0 of z .. z + 63
                uint64_t wz = ~0ull;
                if (first != 0xFFFFFFFFu && !dense) {
                    wz = p0 + (R.ze[first] & 2047u);
                    const uint64_t pl = wz + lane;
                    const uint32_t x = pl - 1 < n ? sym[pl - 1] : 0u;
                    const uint32_t s0q = pl < n ? s0_at(pk, pl - hdr) : 0u;
                    reinterpret_cast<uint8_t *>(R.wx)[lane] = (uint8_t)x;
                    const uint64_t b0 = ballot(s0q & 1u), b1 = ballot(s0q & 2u);
                    if (lane == 0) {
                        R.ws[0] = (uint32_t)b0;
                        R.ws[1] = (uint32_t)(b0 >> 32);
                        R.ws[2] = (uint32_t)b1;
                        R.ws[3] = (uint32_t)(b1 >> 32);
                    }
                }
                if (lane == 0) {
                    R.ver = v;
                    R.first = first;
                    R.zn = rec.zn;
                    R.s0 = rec.s0;
                    R.L = rec.L;
                    R.o0 = rec.o0;
                    R.wz = wz;
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot's LDS writes are done
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) lds_st(&R.j, (uint32_t)j);  // published
            }
        } else {
            // -------------------------------------------------------------- consumer
            int64_t D = 0;         // true offset - no-reset offset, outside the windows
            uint64_t resume = 0;   // symbols below this are inside a window already done
            uint32_t ver = 0;
            uint64_t next_chunk = 0;
            bool stop = false;     // an error or the end inside a window: the walks report it
            uint32_t fall = 0;
#ifdef HC_DEBUG_HOOKS
            // cycles: slot waits, tests, slow hits; counts: subs tested again, skipped by the
            // bitmap, fast hits, slow hits, dense subs
            uint64_t dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PDG_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PDG_ADD(k, t0) (dg[k] += __builtin_amdgcn_s_memtime() - (t0))
#define PDG_CNT(k) (++dg[k])
#else
#define PDG_T(v)
#define PDG_ADD(k, t0)
#define PDG_CNT(k)
#endif
            auto publish = [&]() __attribute__((always_inline)) {
                ++ver;
                if (lane == 0) {
                    vD[ver % 64] = D;
                    vres[ver % 64] = resume;
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) lds_st(&sh_ver, ver);
            };
            for (uint64_t j = 0; j < nsub && !stop; ++j) {
                RSlot &R = ring[j % kRing];
                PDG_T(t_w);
                for (uint32_t spin = 0; lds_ld(&R.j) != (uint32_t)j; ++spin) {
                    if (lds_ld(&sh_quit) || spin > kSpinCap) {  // (a producer gave up: never expected)
                        fall = 1;
                        stop = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                PDG_ADD(0, t_w);
                if (stop) break;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint64_t p0 = hdr + j * kSub;
                const uint64_t o0 = R.o0;
                const uint32_t zn = R.zn, rv = R.ver, rfirst = R.first;
                if (j % kSubPerChunk == 0 && j / kSubPerChunk >= next_chunk) {
                    const uint64_t c = j / kSubPerChunk;
                    if (lane == 0) {
                        C[c].q0 = p0;
                        C[c].o_in = o0 + D;
                        C[c].r_in = R.s0;
                    }
                    next_chunk = c + 1;
                }
                const bool dense = zn == kDense;
                const uint32_t cnt = (uint32_t)((p0 + kSub < n ? p0 + kSub : n) - p0);
                const uint32_t items = dense ? cnt : zn;
                // the producer's test holds while no block start was found since it ran; after
                // one, the bitmap says whether any entry has the residue a start needs now (when
                // every entry is in the full block rows)
                bool skip = rv == ver && rfirst == 0xFFFFFFFFu;
                if (!skip && rv != ver && pow2 && o0 + D + R.L < full_end) {
                    // a start needs (o0 + rel + D) = 0 mod B^2: residue (o0 + rel) = -D
                    const uint32_t want = (uint32_t)((0 - (uint64_t)D) & mask) & 1023u;
                    skip = ((R.bm[want >> 5] >> (want & 31)) & 1u) == 0;
                    if (skip) PDG_CNT(4);
                }
                PDG_T(t_t);
                if (!skip) {
                    PDG_CNT(3);
                    if (dense) PDG_CNT(7);
                    // the batches of 64 entries that can hold a start under (D, resume), lane k
                    // for batch k: entries are sorted by offset, so batch k's offsets span
                    // [first, last] and a start needs one = -(o0 + D) mod B^2 in that range
                    auto batches = [&]() __attribute__((always_inline)) -> uint64_t {
                        const uint32_t nbt = (items + 63) / 64, k = lane;
                        bool maybe = false;
                        if (k < nbt) {
                            const uint32_t ef = R.ze[64 * k], el = R.ze[min(64 * k + 63, items - 1)];
                            const uint32_t rf = ef >> 11, rl = el >> 11;
                            const uint64_t base = o0 + D;
                            maybe = true;
                            if (pow2 && base + rl < full_end) {
                                const uint32_t t = (uint32_t)((0 - base) & mask);
                                maybe = ((t - rf) & (uint32_t)mask) <= rl - rf;
                            }
                            const uint32_t rres = resume <= p0 ? 0u : (resume - p0 >= kSub ? kSub : (uint32_t)(resume - p0));
                            if ((el & 2047u) < rres) maybe = false;  // the whole batch is behind resume
                        }
                        return ballot(maybe);
                    };
                    uint64_t bmask = batches();
                    if (rv == ver && rfirst != 0xFFFFFFFFu) bmask &= ~0ull << (rfirst >> 6);
                    while (bmask && !stop) {
                        const uint32_t bk = (uint32_t)__builtin_ctzll(bmask), b = 64 * bk;
                        const bool ok = b + lane < items;
                        const uint32_t e = ok ? R.ze[b + lane] : 0xFFFFFFFFu;
                        const uint64_t cand = ballot(test(e, ok, p0, o0, D, resume));
                        if (!cand) {
                            bmask &= bmask - 1;
                            continue;
                        }
                        const uint32_t idx = b + (uint32_t)__builtin_ctzll(cand);
                        const uint32_t eL = R.ze[idx];
                        const uint32_t ziL = dense ? 0u : R.zi[idx];
                        const uint64_t z = p0 + (eL & 2047u);
                        const uint64_t oz0 = o0 + (eL >> 11);  // O0(z)
                        const uint64_t o = oz0 + D;
                        // fast path: the window par_z described, inside one block (B^2 bytes),
                        // no chunk start inside it
                        const uint32_t wl = ziL & 63u, wo = ziL >> 19;
                        const uint64_t cz = (z - hdr) / span, cw = (z + wl - 1 - hdr) / span;
                        if (ziL && o < full_end && mask + 1 > wo && cz == cw) {
                            PDG_CNT(5);
                            D += (int64_t)((ziL >> 6) & 8191u) - 4096;
                            resume = z + wl;
                            publish();
                            bmask = batches() & (~0ull << bk);
                            continue;
                        }
                        PDG_CNT(6);
                        PDG_T(t_h);
                        // the true machine from the block start z until it rejoins s0; the
                        // window from the slot (a dense sub-chunk's symbols, or the one the
                        // producer prefetched) while it lasts. Blocks in the full rows hold
                        // B^2 bytes; elsewhere the block's place gives its size.
                        uint64_t ot = o, o0t = oz0, got = 0, want;
                        if (o < full_end) {
                            want = mask + 1;
                        } else {
                            uint64_t bx, by, rl;
                            g.locate(ot, bx, by, rl);
                            want = g.sx(bx) * g.sy(by);
                        }
                        uint32_t u = 0;
                        uint64_t q = z;
                        uint32_t xw = 0, sw0 = 0;  // window: symbols q - 1 + lane, s0 of q + lane
                        uint64_t wbase = ~0ull;
                        auto load_window = [&]() __attribute__((always_inline)) {
                            wbase = q;
                            const uint64_t pl = q + lane;
                            const uint64_t r1 = pl - 1 - p0, r0 = pl - p0;
                            if (dense && pl - 1 >= p0 && r1 < cnt) {
                                xw = reinterpret_cast<const uint8_t *>(R.sx)[r1];
                            } else {
                                xw = pl - 1 < n ? sym[pl - 1] : 0u;
                            }
                            if (dense && r0 < cnt) {
                                sw0 = (R.sp[r0 >> 4] >> (2 * (r0 & 15))) & 3u;
                            } else {
                                sw0 = pl < n ? s0_at(pk, pl - hdr) : 0u;
                            }
                        };
                        if (!dense && R.wz == z) {
                            wbase = z;
                            xw = reinterpret_cast<const uint8_t *>(R.wx)[lane];
                            const uint64_t p0l = (uint64_t)R.ws[1] << 32 | R.ws[0], p1l = (uint64_t)R.ws[3] << 32 | R.ws[2];
                            sw0 = (uint32_t)((p0l >> lane) & 1u) | (uint32_t)(((p1l >> lane) & 1u) << 1);
                        }
                        for (;;) {
                            if (q > z && got == 0) u = 0;  // a block start inside the window
                            if (q >= n) {
                                stop = true;
                                break;
                            }
                            if (q - z >= kWinCap) {
                                fall = 1;
                                stop = true;
                                break;
                            }
                            if (wbase == ~0ull || q - wbase >= 63) load_window();  // (re)load at q
                            const uint32_t s0q = readlane(sw0, (uint32_t)(q - wbase));
                            if (q > z && u == s0q) break;  // rejoined
                            if ((q - hdr) % span == 0 && q > z) {
                                // a chunk start inside the window: its walk runs in from z
                                const uint64_t c = (q - hdr) / span;
                                if (lane == 0) {
                                    C[c].q0 = z;
                                    C[c].o_in = oz0 + D;
                                    C[c].r_in = 0;
                                }
                                next_chunk = c + 1;
                            }
                            const uint32_t x = readlane(xw, (uint32_t)(q - wbase) + 1);
                            const uint32_t xp = readlane(xw, (uint32_t)(q - wbase));
                            const uint32_t lt = u == 3 ? x : 1u;
                            o0t += s0q == 3 ? x : 1u;
                            ot += lt;
                            got += lt;
                            u = fsm_at(fsm_step(x, xp), u);
                            ++q;
                            if (got > want) {  // overshoot: status 13, reported by the walks
                                stop = true;
                                break;
                            }
                            if (got == want) {  // the next block starts at offset ot
                                got = 0;
                                if (ot < full_end) {
                                    want = mask + 1;
                                } else if (ot >= g.total) {  // the last block: leftover is the walks' to report
                                    stop = true;
                                    break;
                                } else {  // the last block row or another geometry
                                    uint64_t bx, by, rl;
                                    g.locate(ot, bx, by, rl);
                                    want = g.sx(bx) * g.sy(by);
                                }
                            }
                        }
                        PDG_ADD(2, t_h);
                        if (stop) break;
                        D = (int64_t)(ot - o0t);
                        resume = q;
                        publish();
                        bmask = batches() & (~0ull << bk);
                    }
                }
                PDG_ADD(1, t_t);
                if (lane == 0) lds_st(&sh_done, (uint32_t)(j + 1));
            }
            if (lane == 0) lds_st(&sh_quit, 1u);
            // chunks past a stop (an error or the stream's end inside a window: the walks before
            // them report it) get a neutral entry; par_fix re-runs them if it ever reaches them
            for (uint64_t c = next_chunk + lane; c < M.nchk; c += 64) {
                C[c].q0 = hdr + c * span;
                C[c].o_in = 0;
                C[c].r_in = 0xFFu;
            }
            if (lane == 0) M.pfall = fall;
#ifdef HC_DEBUG_HOOKS
            if (lane < 8) {
                uint64_t dv = dg[0];
#pragma unroll
                for (uint32_t k = 1; k < 8; ++k) dv = lane == k ? dg[k] : dv;
                M.pdiag[lane] = dv;
            }
#endif
        }
        __syncthreads();
    }
}

// one wave per chunk: the serial process from the predicted entry
__global__ __launch_bounds__(256) void par_walk_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t items = ws.ctr[3];
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < items; t += (uint64_t)gridDim.x * 4) {
        uint32_t i;
        uint64_t j;
        if (!sub_item(a, ws, t, i, j) || j % kSubPerChunk) continue;
        const AMeta &M = ws.meta[i];
        if (M.pfall) continue;
        PChk &C = pchk(ws, M)[j / kSubPerChunk];
        const uint64_t q = M.hdr + j * kSub;
        const uint64_t qe = q + (uint64_t)kSub * kSubPerChunk < M.count ? q + (uint64_t)kSub * kSubPerChunk : M.count;
        BWalk w;
        w.init(M, at<uint8_t>(ws, M.sym), at<uint64_t>(ws, M.starts), lane);
        const uint64_t q0 = C.q0;
        if (q0 > q || q0 < M.hdr || C.r_in > 3) {  // no prediction: par_fix runs the chunk
            if (lane == 0) {
                C.r_q = 0xFFu;
                C.e_lo = ~0ull;
                C.e_hi = 0;
            }
            continue;
        }
        uint64_t o_in = C.o_in;
#ifdef HC_DEBUG_HOOKS
        if (g_par_skew && (j / kSubPerChunk) % 2 == 1) o_in = (o_in + g_par_skew) % (M.w * M.h);
#endif
        w.enter(q0, C.r_in, o_in, q);
        uint32_t r_q = C.r_in;
        uint64_t o_q = o_in;
        int st = 0;
        if (q0 < q) {  // run in from the window's block start (recording nothing before q)
            st = w.run(q, q);
            r_q = st ? 0xFFu : w.r;
            o_q = w.offset();
        }
        if (st == 0) st = w.run(qe, q);
        if (lane == 0) {
            C.r_q = r_q;
            C.o_q = o_q;
            C.st = (uint32_t)st;
            C.r_out = w.r;
            C.o_out = w.offset();
            C.e_lo = w.e_lo;
            C.e_hi = w.e_hi;
        }
    }
}

// one wave per stream: chunk entries against the exact exits before them, 64 chunks at a time
// (lane k: chunk c, its predicted entry against chunk c - 1's exit); the first chunk that differs
// (or every chunk, after a fallback) is re-run here from the exact exit, then the check goes on
// after it; the first error in chunk order is the stream's status.
// A walk from a wrong entry numbers its blocks wrongly, so the entries it wrote (its e_lo..e_hi)
// may belong to blocks of other chunks, whose own walks raced with it. The re-run rewrites only
// the re-run chunk's blocks; afterwards every chunk whose blocks meet such a range is walked once
// more from its exact entry (kept in C by the first pass), which rewrites each entry there with
// its true start (tests/bounds_par_model.py keeps a walk's starts aside until it is verified; the
// GPU pass writes them at once and repairs them here).
__global__ __launch_bounds__(64) void par_fix_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id();
    for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        AMeta &M = ws.meta[i];
        if (M.status || !M.par) continue;
        PChk *C = pchk(ws, M);
        BWalk w;
        w.init(M, at<uint8_t>(ws, M.sym), at<uint64_t>(ws, M.starts), lane);
        const Geo g = w.geo();
        const bool fall = M.pfall != 0;
        const uint64_t nchk = M.nchk, span = (uint64_t)kSub * kSubPerChunk;
        uint32_t r = 0, st = 0;  // the exact process before chunk c
        uint64_t o = 0, reruns = 0, c = 0;
        uint64_t dlo = ~0ull, dhi = 0;  // entries written by walks from wrong entries
        // nchk >= 1: dec_header_kernel sets par only when the stream holds block symbols (an
        // empty body reaches the serial pass, which reports HC_ERR_BLOCK_EOF, transform.cpp:170-174)
        while (c < nchk && !st) {
            const uint64_t cl = c + lane;
            const bool on = cl < nchk;
            const uint32_t r_q = on ? C[cl].r_q : 0u, r_out = on ? C[cl].r_out : 0u, cst = on ? C[cl].st : 0u;
            const uint64_t o_q = on ? C[cl].o_q : 0, o_out = on ? C[cl].o_out : 0;
            // the exit before each lane's chunk: the lane below's (lane 0: the exact one)
            const uint32_t pr = lane_shr1(r_out, r);
            const uint64_t po = (uint64_t)lane_shr1((uint32_t)o_out, (uint32_t)o) |
                                (uint64_t)lane_shr1((uint32_t)(o_out >> 32), (uint32_t)(o >> 32)) << 32;
            // the walk matches the exact process if it entered at the same offset in the same
            // state (at a block start the state is reset either way)
            const bool same = !fall && r_q != 0xFFu && o_q == po && (r_q == pr || g.is_start(po));
            const uint64_t bad = ballot(on && (!same || cst != 0));
            if (!bad) {
                const uint32_t last = (uint32_t)((nchk - c < 64 ? nchk - c : 64) - 1);
                r = readlane(r_out, last);
                o = (uint64_t)readlane((uint32_t)o_out, last) | (uint64_t)readlane((uint32_t)(o_out >> 32), last) << 32;
                c += 64;
                continue;
            }
            const uint32_t L = (uint32_t)__builtin_ctzll(bad);
            c += L;  // chunks c .. c + L - 1 agree and end without an error
            r = readlane(pr, L);
            o = (uint64_t)readlane((uint32_t)po, L) | (uint64_t)readlane((uint32_t)(po >> 32), L) << 32;
            if (readlane((uint32_t)same, L)) {  // an exact chunk that reports an error
                st = readlane(cst, L);
                break;
            }
            ++reruns;  // re-run chunk c from the exact process
            if (!fall && C[c].r_q != 0xFFu && C[c].e_lo <= C[c].e_hi) {
                dlo = min(dlo, C[c].e_lo);
                dhi = max(dhi, C[c].e_hi);
            }
            const uint64_t q = M.hdr + c * span, qe = q + span < M.count ? q + span : M.count;
            w.enter(q, r, o, q);
            st = (uint32_t)w.run(qe, q);
            // the exact entry and exit, for the repair pass
            if (lane == 0) {
                C[c].r_q = r;
                C[c].o_q = o;
                C[c].r_out = w.r;
                C[c].o_out = w.offset();
                C[c].st = st;
            }
            r = w.r;
            o = w.offset();
            ++c;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // lane 0's C[] writes, read back below
        // repair: walk again every chunk whose blocks (those that start between its exact entry
        // and exit offsets) meet the entries a wrong walk wrote
        if (st == 0 && dlo <= dhi) {
            for (uint64_t c0 = 0; c0 < nchk; c0 += 64) {
                const uint64_t cl = c0 + lane;
                bool hit = false;
                if (cl < nchk) {
                    auto ent = [&](uint64_t off) -> uint64_t {
                        if (off >= g.total) return g.nb / M.K;
                        uint64_t bx, by, rel;
                        g.locate(off, bx, by, rel);
                        return (by * g.per_row + bx) / M.K;
                    };
                    const uint64_t lo = ent(C[cl].o_q), hi = ent(C[cl].o_out);
                    hit = lo <= dhi && hi >= dlo;
                }
                for (uint64_t hm = ballot(hit); hm; hm &= hm - 1) {
                    const uint64_t cc = c0 + (uint64_t)__builtin_ctzll(hm);
                    const uint64_t q = M.hdr + cc * span, qe = q + span < M.count ? q + span : M.count;
                    w.enter(q, C[cc].r_q, C[cc].o_q, q);
                    (void)w.run(qe, q);
                }
            }
        }
        if (lane == 0) {
            M.status = (int32_t)st;
            M.preruns = reruns;
        }
    }
}

// transform.cpp:162-187 for one block by one wave: revert its RLE from symbol `pos` with a
// fresh machine, 64 symbols per step (read(p): symbol p + lane), handing every output byte
// (block-relative index q in scan order, value) to place(); returns the block's end. A count
// repeats the literal before it: literals are placed by their own lanes, each count's run
// (up to 255 bytes) by the whole wave, 64 bytes at a time.
// Idx: the block-relative byte index type (uint32_t for the tile path's blocks of <= 2^14 bytes)
template <class Idx = uint64_t, class Read, class Place>
__device__ __forceinline__ uint64_t revert_block(Read &&read, uint64_t pos, uint64_t count, Idx want,
                                                 Place place, uint32_t lane)
{
    Idx got = 0;
    uint32_t r = 0, last = 0;
    while (got < want && pos < count) {  // (the bounds pass proved the block whole)
        const uint32_t xs = read(pos);
        const uint32_t pr = lane_shr1(xs, last);
        const uint32_t inc = fsm_scan(xs == pr ? kFsmEq : kFsmNe);
        const uint32_t s = fsm_at(lane_shr1(inc, kFsmId), r);
        const uint32_t len = s == 3 ? xs : 1u;
        const uint32_t val = s == 3 ? pr : xs;
        const uint32_t acc = wave_sum_incl(len);
        const Idx need = want - got;
        const uint64_t hit = ballot((Idx)acc >= need);
        const uint32_t L = hit ? (uint32_t)__builtin_ctzll(hit) : 63u;  // last lane of this block
        const bool mine = lane <= L;
        const Idx q0 = got + acc - len;
        if (mine && len == 1) place(q0, val);
        for (uint64_t runs = ballot(mine && len > 1); runs; runs &= runs - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(runs);
            const uint32_t n = readlane(len, l), v = readlane(val, l);
            const Idx b = got + readlane(acc, l) - n;
            for (uint32_t j0 = 0; j0 < n; j0 += 64)
                if (j0 + lane < n) place(b + j0 + lane, v);
        }
        got += readlane(acc, L);
        r = fsm_at(readlane(inc, L), r);
        last = readlane(xs, L);
        pos += L + 1;
    }
    return pos;
}

// A wave's window on a symbol stream read in order: the symbols below `hi` (a multiple of 256)
// sit in a 1 KB LDS ring, the next kPF x 256 are in flight in registers (one dword per lane
// each), so the revert's 64-symbol steps read LDS, not HBM, and a refill waits on a load issued
// kPF refills (4 kPF steps) earlier: with one in flight, the refills waited on HBM latency.
#ifndef HC_RING_PF
#define HC_RING_PF 1
#endif
struct SymRing {
    static constexpr uint32_t kPF = HC_RING_PF;
    uint8_t *R;
    const uint32_t *sw;  // the symbols as dwords (the slab is 16-aligned)
    uint64_t nsym, hi;
    uint32_t pf[kPF], lane;
    __device__ __forceinline__ uint32_t fetch(uint64_t at) const
    {
        const uint64_t o = at + 4 * lane;
        return o < nsym ? sw[o >> 2] : 0u;  // (a dword starting below nsym: inside the slack)
    }
    __device__ __forceinline__ void start(uint64_t pos)
    {
        const uint64_t base = pos & ~255ull;
        uint32_t q[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) q[k] = fetch(base + 256 * k);
        hi = base + 1024;
#pragma unroll
        for (uint32_t k = 0; k < kPF; ++k) pf[k] = fetch(hi + 256 * k);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            *reinterpret_cast<uint32_t *>(R + ((base + 256 * k + 4 * lane) & 1023)) = q[k];
        __builtin_amdgcn_wave_barrier();
    }
    // symbols p + 4 lane .. p + 4 lane + 3 as one dword (byte k: symbol p + 4 lane + k), from two
    // aligned ring dwords (p + 260 <= hi afterwards)
    __device__ __forceinline__ uint32_t read4(uint64_t p)
    {
        while (p + 260 > hi) {
            *reinterpret_cast<uint32_t *>(R + ((hi + 4 * lane) & 1023)) = pf[0];
#pragma unroll
            for (uint32_t k = 0; k + 1 < kPF; ++k) pf[k] = pf[k + 1];
            pf[kPF - 1] = fetch(hi + 256 * kPF);
            hi += 256;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t a = (uint32_t)p + 4 * lane;
        const uint32_t w0 = *reinterpret_cast<const uint32_t *>(R + (a & 1020u));
        const uint32_t w1 = *reinterpret_cast<const uint32_t *>(R + ((a + 4) & 1020u));
        return __builtin_amdgcn_alignbyte(w1, w0, a & 3u);
    }
    // symbol p + lane (p + 64 <= hi afterwards; p >= hi - 1024 by construction)
    __device__ __forceinline__ uint32_t operator()(uint64_t p)
    {
        while (p + 64 > hi) {
            *reinterpret_cast<uint32_t *>(R + ((hi + 4 * lane) & 1023)) = pf[0];
#pragma unroll
            for (uint32_t k = 0; k + 1 < kPF; ++k) pf[k] = pf[k + 1];
            pf[kPF - 1] = fetch(hi + 256 * kPF);
            hi += 256;
        }
        __builtin_amdgcn_wave_barrier();
        return R[(p + lane) & 1023];
    }
};

// transform.cpp:162-187 for a whole block (B a power of two, B x B bytes) of the tile path, 256
// symbols per step: each lane takes 4 consecutive symbols (one ring dword), composes their
// transitions, and one wave scan of the composed functions and one of the lanes' output lengths
// serve all four (64 symbols per step paid two scans and four lane reads per 64). Literals are
// placed by their lanes (a lane past the block end writes to the image's unused pad byte), each
// count's run by the whole wave. The bounds pass proved the block whole, so its end lies in the
// stream and the last step's lanes past it are never placed.
struct RevChain {
    SymRing rd;
    uint32_t *Mk;  // the wave's 128 run marks (64 + a discard slot per lane)
    uint64_t pos;
    uint32_t got, want, r, last;
    uint32_t tb, sl, so, lg, bm;  // T byte of element q: tb + (q >> lg) * sl + (q & bm) * so
    // (24-bit multiplies: v_mul_lo_u32 issues at a quarter of the rate, 8 of them per step)
    __device__ __forceinline__ uint32_t at(uint32_t q) const { return tb + __umul24(q >> lg, sl) + __umul24(q & bm, so); }
    __device__ __forceinline__ void begin(uint64_t p, uint32_t b32, uint32_t x0, uint32_t y0, bool horiz)
    {
        pos = p;
        got = 0;
        want = b32 * b32;
        r = 0;
        last = 0;
        lg = (uint32_t)__builtin_ctz(b32);
        bm = b32 - 1;
        sl = horiz ? kDS : 1u;
        so = horiz ? 1u : kDS;
        tb = y0 * kDS + x0;
        rd.start(p);
    }
    __device__ __forceinline__ bool live() const { return got < want; }
    __device__ __forceinline__ void step(uint8_t *T, uint32_t lane)
    {
        constexpr uint32_t kPad = kDS - 1;  // row 0's last byte: outside every row's 128 bytes
        const uint32_t w = rd.read4(pos);
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) x[k] = (w >> (8 * k)) & 255u;
        const uint32_t p0 = lane_shr1(x[3], last);
        uint32_t f[4];
        f[0] = x[0] == p0 ? kFsmEq : kFsmNe;
#pragma unroll
        for (uint32_t k = 1; k < 4; ++k) f[k] = x[k] == x[k - 1] ? kFsmEq : kFsmNe;
        const uint32_t F = fsm_then(f[3], fsm_then(f[2], fsm_then(f[1], f[0])));
        const uint32_t inc = fsm_scan(F);
        uint32_t st = fsm_at(lane_shr1(inc, kFsmId), r);
        uint32_t len[4], val[4], c[4], cum = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t pk = k ? x[k - 1] : p0;
            len[k] = st == 3 ? x[k] : 1u;
            val[k] = st == 3 ? pk : x[k];
            cum += len[k];
            c[k] = cum;
            st = fsm_at(f[k], st);
        }
        const uint32_t acc = wave_sum_incl(cum), base = acc - cum + got;
        const uint64_t hit = ballot(acc + got >= want);
        const uint32_t L = hit ? (uint32_t)__builtin_ctzll(hit) : 64u;
        // in lane L the block's last symbol: the first k whose output reaches `want`
        const uint32_t kx = base + c[0] >= want ? 0u : base + c[1] >= want ? 1u : base + c[2] >= want ? 2u : 3u;
        const uint32_t kL = hit ? readlane(kx, L) : 3u;
        const uint32_t lim = lane < L ? 4u : (lane == L ? kL + 1 : 0u);  // this lane's symbols in the block
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t q = base + c[k] - 1;
            const bool lit = k < lim && len[k] == 1;
            T[lit ? at(q) : kPad] = (uint8_t)val[k];
        }
        // Runs, all of the step's at once. A count follows three literals, so counts sit >= 4
        // symbols apart: a lane holds at most one (rl bytes of rv from block byte rq). Lane j of a
        // 64-byte chunk of the runs' concatenated bytes (run space) takes the run that starts last
        // at or before it: each run marks its start with key (rq - rs) << 8 | rv, rs its run-space
        // start, and a max-scan of the marks finds it (the keys grow with the runs: >= 3 literal
        // bytes lie between two runs), the byte then sits at block byte j + (key >> 8).
        uint32_t rl = 0, rq = 0, rv = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const bool run = k < lim && len[k] > 1;
            rl = run ? len[k] : rl;
            rq = run ? base + c[k] - len[k] : rq;
            rv = run ? val[k] : rv;
        }
        if (ballot(rl != 0)) {
            const uint32_t rin = wave_sum_incl(rl), rs = rin - rl, rt = readlane(rin, 63);
            const uint32_t key = (rq - rs) << 8 | rv;
            uint32_t carry = 0;  // the run covering the previous chunk's last byte
            for (uint32_t j0 = 0; j0 < rt; j0 += 64) {
                Mk[lane] = lane ? 0u : carry;
                const uint32_t o = rs - j0;
                Mk[rl != 0 && o < 64 ? o : 64 + lane] = key;
                __builtin_amdgcn_wave_barrier();
                const uint32_t kk = wave_scan(Mk[lane], 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
                __builtin_amdgcn_wave_barrier();
                carry = readlane(kk, 63);
                const uint32_t q = j0 + lane + (kk >> 8);
                T[j0 + lane < rt ? at(q) : kPad] = (uint8_t)kk;
            }
        }
        if (hit) {
            got = want;
        } else {
            got += readlane(acc, 63);
            r = fsm_at(readlane(inc, 63), r);
            last = readlane(x[3], 63);
            pos += 256;
        }
    }
};

// transform.cpp:191-216 for blocks of B = 8..128 (mode 0): one workgroup per tile, the blocks
// reverted into an LDS image of the tile, which then leaves as whole rows. The bounds pass
// records every block's start (mode 0), so the blocks are independent: wave wv takes blocks
// wv, wv + 4, .. of the tile (RevChain, 256 symbols per step); their starts and scan orders are
// loaded in one round trip per tile (lane m: block wv + 4 m). Tiles with partial blocks (matrix
// edges) take revert_block, one block at a time.
#ifndef HC_UNB_WPE
#define HC_UNB_WPE 7
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HC_UNB_WPE))) void unblock_tile_kernel(DecArgs a, Ws ws)
{
    __shared__ uint8_t T[kTile * kDS];
    __shared__ uint32_t ring[4][256];
    __shared__ uint32_t marks[4][128];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t ntiles = ws.ctr[2];
    RevChain ca;
    ca.rd.R = reinterpret_cast<uint8_t *>(ring[wv]);
    ca.Mk = marks[wv];
    ca.rd.lane = lane;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tid = tid_here(), lane = tid & 63, wv = tid >> 6;
        (void)tid;
        ca.rd.lane = lane;
        const uint32_t i = find_item(ws.idx[2], a.n, t, ws.ctr[8 + 2]);
        const AMeta &M = ws.meta[i];
        if (M.status || M.mode != 0) continue;  // (uniform over the workgroup)
        const uint64_t W = M.w, H = M.h, B = M.B;
        const uint64_t ntx = cdiv(W, kTile), local = t - ws.idx[2][i];
        const uint64_t tix = local % ntx, tx0 = tix * kTile, ty0 = (local / ntx) * kTile;
        const uint32_t tw = (uint32_t)(W - tx0 < kTile ? W - tx0 : kTile);
        const uint32_t th = (uint32_t)(H - ty0 < kTile ? H - ty0 : kTile);
        const uint32_t b32 = (uint32_t)B;
        const uint32_t nbx = (tw + b32 - 1) / b32, nby = (th + b32 - 1) / b32, nblk = nbx * nby;
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        const uint64_t *starts = at<uint64_t>(ws, M.starts);
        const uint64_t per_row = cdiv(W, B);
        // The wave's blocks wv, wv + 4, .. (lane m: block wv + 4 m, <= 64 of them): each lane loads
        // its block's start and scan order, one round trip per tile. (Whole block rows per wave,
        // one ring fill per row, measured slower: 3.53 vs 3.33 ms on A512.)
        auto block_of = [&](uint32_t m, uint32_t &by, uint32_t &bx) __attribute__((always_inline)) {
            const uint32_t b = wv + 4 * m;
            by = b / nbx;
            bx = b - by * nbx;
        };
        uint64_t bpos = 0;
        uint32_t bh = 0;
        {
            uint32_t by, bx;
            block_of(lane, by, bx);
            if (by < nby) {
                const uint64_t kl = (ty0 / B + by) * per_row + tx0 / B + bx;
                bpos = starts[kl];
                bh = (sym[24 + kl / 8] >> (7 - kl % 8)) & 1;
            }
        }
        auto pos_of = [&](uint32_t m) __attribute__((always_inline)) {
            return (uint64_t)readlane((uint32_t)bpos, m) | (uint64_t)readlane((uint32_t)(bpos >> 32), m) << 32;
        };
        ca.rd.sw = reinterpret_cast<const uint32_t *>(sym);
        ca.rd.nsym = M.count;
        const uint32_t nm = nblk > wv ? (nblk - wv + 3) / 4 : 0u;
        if (tw % b32 == 0 && th % b32 == 0) {  // (uniform) whole blocks only
            for (uint32_t m = 0; m < nm; ++m) {
                uint32_t by, bx;
                block_of(m, by, bx);
                ca.begin(pos_of(m), b32, bx * b32, by * b32, readlane(bh, m) != 0);
                while (ca.live()) ca.step(T, lane);
            }
        } else {
            SymRing &rd = ca.rd;
            for (uint32_t m = 0; m < nm; ++m) {
                uint32_t by, bx;
                block_of(m, by, bx);
                const uint32_t x0 = bx * b32, y0 = by * b32;
                const uint32_t sx = tw - x0 < b32 ? tw - x0 : b32, sy = th - y0 < b32 ? th - y0 : b32;
                const bool horiz = readlane(bh, m) != 0;
                const uint32_t inner = horiz ? sx : sy;
                const uint64_t pos = pos_of(m);
                rd.start(pos);
                const float inv = 1.0f / (float)inner;
                auto place = [&](uint32_t q, uint32_t v) {
                    const uint32_t a1 = div_small((uint32_t)q, inner, inv), b1 = (uint32_t)q - a1 * inner;
                    T[(y0 + (horiz ? a1 : b1)) * kDS + x0 + (horiz ? b1 : a1)] = (uint8_t)v;
                };
                revert_block<uint32_t>(rd, pos, M.count, sx * sy, place, lane);
            }
        }
        lds_barrier();
        uint8_t *mat = a.out + a.out_offs[i];
        const uint32_t nd = (tw + 3) / 4;
        for (uint32_t it = tid; it < th * nd; it += 256) {
            const uint32_t r = it / nd, d = it - r * nd;
            uint8_t *dst = mat + (ty0 + r) * W + tx0 + 4 * d;
            const uint32_t v = *reinterpret_cast<const uint32_t *>(T + r * kDS + 4 * d);
            if (4 * d + 4 <= tw) {
                typedef uint32_t u32u __attribute__((aligned(1)));
                *reinterpret_cast<u32u *>(dst) = v;
            } else {
                for (uint32_t k = 0; 4 * d + k < tw; ++k) dst[k] = (uint8_t)(v >> (8 * k));
            }
        }
        lds_barrier();
    }
}

// modes 1 and 2: the blocks of one group per wave, scattered straight to memory
__global__ __launch_bounds__(256) void unblock_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t items = ws.ctr[0];
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wv; t < items; t += (uint64_t)gridDim.x * 4) {
        const uint32_t i = find_item(ws.idx[0], a.n, t, ws.ctr[8 + 0]);
        const AMeta &M = ws.meta[i];
        if (M.status || M.mode == 0) continue;
        const uint64_t g = t - ws.idx[0][i];
        const uint8_t *sym = at<uint8_t>(ws, M.sym);
        uint64_t pos = at<uint64_t>(ws, M.starts)[g];
        uint8_t *mat = a.out + a.out_offs[i];
        const uint64_t W = M.w;
        const uint64_t kb = g * M.K, ke = kb + M.K < M.nb ? kb + M.K : M.nb;
        for (uint64_t k = kb; k < ke; ++k) {
            uint64_t x0, y0, sx, sy;
            block_size(M, k, &x0, &y0, &sx, &sy);
            const bool horiz = (sym[24 + k / 8] >> (7 - k % 8)) & 1;
            const uint64_t inner = horiz ? sx : sy, want = sx * sy;
            const bool small = want < (1u << 24);
            const float inv = 1.0f / (float)inner;
            auto place = [&](uint64_t q, uint32_t v) {
                const uint64_t a1 = small ? div_small((uint32_t)q, (uint32_t)inner, inv) : q / inner;
                const uint64_t b1 = q - a1 * inner;
                mat[(y0 + (horiz ? a1 : b1)) * W + x0 + (horiz ? b1 : a1)] = (uint8_t)v;
            };
            pos = revert_block([&](uint64_t p) -> uint32_t { return sym[p + lane]; }, pos, M.count, want, place, lane);
        }
    }
}

// transform.cpp:231-239 (prefix sum mod 256 over the linear matrix) in 16 KB chunks:
// per-chunk byte sums, a per-stream scan of those, then the chunks' prefix sums
// 16-byte vector of dwords at any 4-aligned address (diff revert loads / stores)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
__global__ __launch_bounds__(256) void chunk_sum_kernel(DecArgs a, Ws ws)
{
    __shared__ uint32_t red[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t items = ws.ctr[1];
    for (uint64_t t = blockIdx.x; t < items; t += gridDim.x) {
        const uint32_t i = find_item(ws.idx[1], a.n, t, ws.ctr[8 + 1]);
        const AMeta &M = ws.meta[i];
        const uint64_t c = t - ws.idx[1][i], n = M.w * M.h;
        const uint64_t b = c * kChunk, e = b + kChunk < n ? b + kChunk : n;
        const uint8_t *mat = a.out + a.out_offs[i] + b;  // this chunk (out_offs 4-aligned)
        const uint32_t len = (uint32_t)(e - b);
        uint32_t s = 0;
        if (len == kChunk) {  // 16-byte loads, 4 per thread
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const u32x4 q = *reinterpret_cast<const u32x4 *>(mat + 4096 * k + 16 * tid);
                s = __builtin_amdgcn_sad_u8(q.x, 0u, s);
                s = __builtin_amdgcn_sad_u8(q.y, 0u, s);
                s = __builtin_amdgcn_sad_u8(q.z, 0u, s);
                s = __builtin_amdgcn_sad_u8(q.w, 0u, s);
            }
        } else {
            for (uint32_t k = 4 * tid; k < len; k += 1024) {
                uint32_t w = *reinterpret_cast<const uint32_t *>(mat + k);
                if (k + 4 > len) w &= 0xFFFFFFFFu >> (8 * (k + 4 - len));
                s = __builtin_amdgcn_sad_u8(w, 0u, s);
            }
        }
        for (uint32_t d = 32; d; d >>= 1) s += __shfl_down(s, d, 64);
        if ((tid & 63) == 0) red[tid >> 6] = s;
        lds_barrier();
        if (tid == 0) at<uint8_t>(ws, M.csum)[c] = (uint8_t)(red[0] + red[1] + red[2] + red[3]);
        lds_barrier();
    }
}

__global__ __launch_bounds__(64) void chunk_scan_kernel(DecArgs a, Ws ws)
{
    const uint32_t lane = lane_id();
    for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        const AMeta &M = ws.meta[i];
        if (M.status || !M.chunks) continue;
        uint8_t *cs = at<uint8_t>(ws, M.csum);
        uint32_t carry = 0;
        for (uint64_t b = 0; b < M.chunks; b += 64) {
            const bool ok = b + lane < M.chunks;
            const uint32_t v = ok ? cs[b + lane] : 0u;
            const uint32_t acc = wave_sum_incl(v);
            if (ok) cs[b + lane] = (uint8_t)(carry + acc - v);  // exclusive
            carry += readlane(acc, 63);
        }
    }
}

// one 16 KB chunk per workgroup as four 4 KB segments; in each, thread t holds 16 bytes at 16 t
// (coalesced 16-byte loads and stores): byte prefix sums inside each dword (two shifted bytewise
// adds), carried along the thread's 4 dwords; the four segments' thread totals packed one per
// byte and scanned bytewise across the workgroup (mod 256 per byte, no carries between them);
// the segments carried one after another from the chunks before (chunk_scan_kernel)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void undiff_kernel(DecArgs a, Ws ws)
{
    __shared__ uint32_t part[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t items = ws.ctr[1];
    for (uint64_t t = blockIdx.x; t < items; t += gridDim.x) {
        const uint32_t i = find_item(ws.idx[1], a.n, t, ws.ctr[8 + 1]);
        const AMeta &M = ws.meta[i];
        const uint64_t c = t - ws.idx[1][i], n = M.w * M.h;
        const uint64_t b = c * kChunk, e64 = b + kChunk < n ? b + kChunk : n;
        uint8_t *mat = a.out + a.out_offs[i] + b;  // this chunk
        const uint32_t e = (uint32_t)(e64 - b);     // its length
        auto run_chunk = [&](auto full) __attribute__((always_inline)) {
            constexpr bool kFull = decltype(full)::value;
            const uint32_t c0 = at<uint8_t>(ws, M.csum)[c];
            uint32_t w[16];
    #pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t o = 4096 * k + 16 * tid;
                if (kFull || o + 16 <= e) {
                    const u32x4 q = *reinterpret_cast<const u32x4 *>(mat + o);
                    w[4 * k] = q.x;
                    w[4 * k + 1] = q.y;
                    w[4 * k + 2] = q.z;
                    w[4 * k + 3] = q.w;
                } else {
    #pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t od = o + 4 * d;
                        w[4 * k + d] = od < e ? *reinterpret_cast<const uint32_t *>(mat + od) : 0u;
                        if (od < e && od + 4 > e) w[4 * k + d] &= 0xFFFFFFFFu >> (8 * (od + 4 - e));
                    }
                }
            }
            uint32_t tot = 0;  // byte k: this thread's total of segment k
    #pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t run = 0;
    #pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t y = add8(w[4 * k + d], w[4 * k + d] << 8);
                    y = add8(y, y << 16);
                    w[4 * k + d] = add8(y, run * 0x01010101u);
                    run = w[4 * k + d] >> 24;
                }
                tot |= run << (8 * k);
            }
            const uint32_t acc = wave_scan(tot, 0u, [](uint32_t x, uint32_t y) { return add8(x, y); });
            if (lane == 63) part[wv] = acc;
            lds_barrier();
            uint32_t before = sub8(acc, tot);  // the threads before, per segment
            uint32_t all = 0;                  // the segments' totals
    #pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t pk = part[k];
                if (k < wv) before = add8(before, pk);
                all = add8(all, pk);
            }
            uint32_t seg = c0;  // carry into segment k: the chunks before + segments 0..k-1
    #pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t add = ((seg + (before >> (8 * k))) & 0xFFu) * 0x01010101u;
                seg += all >> (8 * k);
                const uint32_t o = 4096 * k + 16 * tid;
                u32x4 q;
                q.x = add8(w[4 * k], add);
                q.y = add8(w[4 * k + 1], add);
                q.z = add8(w[4 * k + 2], add);
                q.w = add8(w[4 * k + 3], add);
                if (kFull || o + 16 <= e) {
                    *reinterpret_cast<u32x4 *>(mat + o) = q;
                } else {
                    const uint32_t v4[4] = {q.x, q.y, q.z, q.w};
    #pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t od = o + 4 * d;
                        if (od + 4 <= e) {
                            *reinterpret_cast<uint32_t *>(mat + od) = v4[d];
                        } else if (od < e) {  // 1..3 bytes
                            mat[od] = (uint8_t)v4[d];
                            if (od + 1 < e) mat[od + 1] = (uint8_t)(v4[d] >> 8);
                            if (od + 2 < e) mat[od + 2] = (uint8_t)(v4[d] >> 16);
                        }
                    }
                }
            }
        };
        if (e == kChunk) run_chunk(std::true_type{});
        else run_chunk(std::false_type{});
        lds_barrier();
    }
}

__global__ void dec_final_kernel(DecArgs a, Ws ws)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const AMeta &M = ws.meta[i];
    a.status[i] = M.status;
    if (M.status == 0) a.out_lens[i] = M.w * M.h;
    else if (M.status != HC_ERR_CAPACITY) a.out_lens[i] = 0;
}

// Persistent grids: exactly the workgroups the device holds at once (CUs x resident workgroups
// per CU at this kernel's LDS / VGPR use), so no workgroup waits for a second round.
template <class Kernel>
unsigned resident_grid(Kernel k, unsigned threads)
{
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, (int)threads, 0) != hipSuccess || cus <= 0 ||
        per <= 0)
        return kGrid;
    return (unsigned)(cus * per);
}

}  // namespace

uint64_t adapt_encode_work_bound(uint64_t total_in, uint32_t n)
{
    // per matrix of L bytes: cost words <= L/3, tile summaries <= 0.19 L, u64 block offsets
    // <= 8 (3L/64 + 1), symbols <= 1.41 L + 42
    return ws_header(n) + 5 * (total_in / 2) + 5 + 176ull * n + 4096;
}

uint64_t adapt_decode_work_bound(uint64_t total_in, uint64_t total_out, uint32_t n)
{
    // symbols <= 8 per payload byte (+64 slack); u64 block starts <= 8 (out_cap / 32 + 16) (see
    // group_entries_bound); chunk sums out_cap / 16384
    // + the parallel boundary pass: per symbol of the streams that take it, the Z entries and
    // their window info (8 kZcap / kSub bytes: 4 at kZcap 1024), packed s0 0.25, records; 4992
    // bytes of rounding per stream
    constexpr uint64_t kPar8 = (8 * (8 * kZcap + kSub / 4 + 64) + kSub - 1) / kSub;  // per 8 symbols
    uint64_t tiny = 0;
#ifdef HC_DEBUG_HOOKS
    // the debug threshold below 2^20 symbols (hc_debug_set_par_min) sends tiny streams through
    // the pass: each may need a whole sub-chunk's records, which the per-symbol term does not cover
    if (g_par_min_host < kParMin) tiny = (8ull * kZcap + kSub / 4 + 256) * n;
#endif
    return ws_header(n) + (8 + kPar8) * total_in + total_out / 4 + total_out / kChunk + 4992ull * n + tiny + 4096;
}

// Diagnostic stage clock (debug build only, hc_debug_stage_clock / hc_debug_stage_times): when
// on, the batched adaptive calls record a HIP event on their stream after every stage, so a
// caller can read each stage's time of its thread's last call (bench.py reports them per stage).
// Per thread: concurrent calls from several threads keep separate clocks.
#ifdef HC_DEBUG_HOOKS
struct StageClock {
    bool on = false;
    bool made = false;
    int n = 0;
    const char *name[32];
    hipEvent_t ev[33];
    void start(hipStream_t st)
    {
        if (!on) return;
        n = 0;
        if (!made) {
            for (auto &e : ev)
                if (hipEventCreate(&e) != hipSuccess) {
                    on = false;
                    return;
                }
            made = true;
        }
        (void)hipEventRecord(ev[0], st);
    }
    void mark(const char *nm, hipStream_t st)
    {
        if (!on || n >= 32) return;
        name[n] = nm;
        (void)hipEventRecord(ev[++n], st);
    }
};
static thread_local StageClock g_clock;
#else
struct StageClock {  // the shipping build: no clock, nothing recorded
    void start(hipStream_t) const {}
    void mark(const char *, hipStream_t) const {}
};
static constexpr StageClock g_clock{};
#endif

hipError_t adapt_encode_batch(const Batch &b, const uint64_t *widths, void *work, uint64_t work_bytes,
                              hipStream_t st)
{
    if (b.n == 0) return hipSuccess;
    const Ws ws = carve(work, work_bytes, b.n);
    const EncArgs a{b.in, b.in_offs, b.in_lens, widths, b.n, (b.flags & HC_FLAG_DIFF) ? 1u : 0u};
    g_clock.start(st);
    enc_plan_kernel<<<1, 1024, 0, st>>>(a, ws);
    g_clock.mark("enc_plan", st);
    tile_cost_kernel<<<resident_grid(tile_cost_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("tile_cost", st);
    big_cost_kernel<<<resident_grid(big_cost_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("big_cost", st);
    choose_kernel<<<b.n < kGrid ? b.n : kGrid, 256, 0, st>>>(a, ws);
    g_clock.mark("choose", st);
    emit_tile_kernel<<<resident_grid(emit_tile_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("emit_tile", st);
    emit_big_kernel<<<resident_grid(emit_big_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("emit_big", st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    Batch f = b;
    f.in = ws.base;
    f.in_offs = ws.sym_offs;
    f.in_lens = ws.sym_lens;
    f.flags = (b.flags & HC_FLAG_DIFF) | HC_FLAG_ADAPT;
    e = launch_encode(f, SRC_SYMBOLS, st);
    if (e != hipSuccess) return e;
    g_clock.mark("fgk_encode", st);
    status_fix_kernel<<<(b.n + 255) / 256, 256, 0, st>>>(ws, b.n, b.status, b.out_lens);
    g_clock.mark("status_fix", st);
    return hipGetLastError();
}

hipError_t adapt_decode_batch(const Batch &b, void *work, uint64_t work_bytes, hipStream_t st)
{
    if (b.n == 0) return hipSuccess;
    const Ws ws = carve(work, work_bytes, b.n);
    const DecArgs a{b.in, b.in_offs, b.in_lens, b.n, b.out, b.out_offs, b.out_caps, b.out_lens, b.status};
    g_clock.start(st);
    dec_plan_kernel<<<1, 1024, 0, st>>>(a, ws);
    g_clock.mark("dec_plan", st);
    Batch f = b;
    f.in_lens = ws.lens2;
    f.out = ws.base;
    f.out_offs = ws.sym_offs;
    f.out_caps = ws.sym_caps;
    f.out_lens = ws.sym_lens;
    hipError_t e = launch_decode(f, DST_SYMBOLS, st);
    if (e != hipSuccess) return e;
    g_clock.mark("fgk_decode", st);
    dec_header_kernel<<<1, 1024, 0, st>>>(a, ws);
    g_clock.mark("dec_header", st);
    bounds_kernel<<<resident_grid(bounds_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("bounds", st);
    // the parallel boundary pass for the streams of many block symbols (none: every launch
    // finds no work item and returns)
    const unsigned per_stream = b.n < kGrid ? b.n : kGrid;
    par_fsm_kernel<<<resident_grid(par_fsm_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("par_fsm", st);
    par_entry_kernel<<<per_stream, 64, 0, st>>>(a, ws);
    g_clock.mark("par_entry", st);
    par_z_kernel<<<resident_grid(par_z_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("par_z", st);
    par_scan_kernel<<<per_stream, 64 * (kProd + 1), 0, st>>>(a, ws);
    g_clock.mark("par_scan", st);
    par_walk_kernel<<<resident_grid(par_walk_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("par_walk", st);
    par_fix_kernel<<<per_stream, 64, 0, st>>>(a, ws);
    g_clock.mark("par_fix", st);
    unblock_tile_kernel<<<resident_grid(unblock_tile_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("unblock_tile", st);
    unblock_kernel<<<resident_grid(unblock_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("unblock", st);
    chunk_sum_kernel<<<resident_grid(chunk_sum_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("chunk_sum", st);
    chunk_scan_kernel<<<b.n < kGrid ? b.n : kGrid, 64, 0, st>>>(a, ws);
    g_clock.mark("chunk_scan", st);
    undiff_kernel<<<resident_grid(undiff_kernel, 256), 256, 0, st>>>(a, ws);
    g_clock.mark("undiff", st);
    dec_final_kernel<<<(b.n + 255) / 256, 256, 0, st>>>(a, ws);
    g_clock.mark("dec_final", st);
    return hipGetLastError();
}

}  // namespace hc

#ifdef HC_DEBUG_HOOKS
extern "C" int hc_debug_set_par_skew(uint64_t bytes)
{
    // 0: off; else every odd chunk of the parallel boundary pass walks from a wrong entry
    return hipMemcpyToSymbol(HIP_SYMBOL(hc::g_par_skew), &bytes, sizeof(bytes)) == hipSuccess ? 0 : HC_ERR_DEVICE;
}

extern "C" int hc_debug_set_par_min(uint64_t symbols)
{
    // block symbols from which an adaptive stream's boundaries take the parallel pass
    hc::g_par_min_host = symbols;
    return hipMemcpyToSymbol(HIP_SYMBOL(hc::g_par_min), &symbols, sizeof(symbols)) == hipSuccess ? 0 : HC_ERR_DEVICE;
}

extern "C" int hc_debug_stage_clock(int on)
{
    hc::g_clock.on = on != 0;
    hc::g_clock.n = 0;
    return 0;
}

// the stages of the last batched adaptive call: names joined by '\n' into names (NUL-ended,
// truncated to names_len), milliseconds into ms[0..max); returns the number of stages (waits for
// the last one), or -1 if the clock is off or an event query fails
extern "C" int hc_debug_stage_times(char *names, int names_len, float *ms, int max)
{
    hc::StageClock &c = hc::g_clock;
    if (!c.on) return -1;
    if (c.n && hipEventSynchronize(c.ev[c.n]) != hipSuccess) return -1;
    int len = 0;
    for (int k = 0; k < c.n && k < max; ++k) {
        if (hipEventElapsedTime(&ms[k], c.ev[k], c.ev[k + 1]) != hipSuccess) return -1;
        for (const char *p = c.name[k]; *p && len + 2 < names_len; ++p) names[len++] = *p;
        if (len + 1 < names_len) names[len++] = '\n';
    }
    if (names_len > 0) names[len < names_len ? len : names_len - 1] = 0;
    return c.n;
}

#endif  // HC_DEBUG_HOOKS

#ifdef HC_TC_PROF
extern "C" int hc_debug_tc_prof(unsigned long long *out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hc::g_tc_prof), sizeof(unsigned long long) * 16) != hipSuccess) return 70;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hc::g_tc_prof), z, sizeof(z)) != hipSuccess) return 70;
    }
    return 0;
}
#endif
