// hc_fgk.hip — FGK adaptive-Huffman encode / decode for gfx950, one stream per wavefront.
//
// Reference: huffman.cpp:23-217 (HuffTree), transform.cpp:363-406 (applyHuffman /
// revertHuffman), fused with transform.cpp:220-292 (diff model, MNP-5 RLE and their inverses)
// and the header / bit packing of headers.cpp:107-125 and main.cpp:39-128.
//
// Design:
//  * The FGK stream is serial, so parallelism comes from the batch: each 64-lane wavefront owns
//    one stream, four wavefronts per 256-thread workgroup, 8 workgroups (32 waves) per CU.
//  * The tree lives in LDS in the implicit slot form of SURVEY.md Appendix A.5: position p in
//    0..512 carries the reference's node number p (root = 512), siblings are (2k, 2k+1), code
//    bit = p & 1, weights non-decreasing in p. Per position one packed word
//    weight << 10 | parent ("narrow", <= 2^22-2 symbols) or a 32-bit weight plus a separate
//    parent array ("wide").
//  * Per update level ONE lane-parallel LDS read fetches the words of positions s..s+63; a
//    64-bit ballot of "weight == w[s]" is a prefix mask (weights sorted), so its trailing-ones
//    count gives the block leader of huffman.cpp:157-184 (highest number with equal weight)
//    in one step.
//  * All control state (positions, bit accumulators, run-length FSM) is wave-uniform and lives
//    in SGPRs. To keep the compiler from turning it into exec-masked VGPR code, the hot loops
//    contain NO lane-divergent control flow: a store "from lane 0 only" is an all-lane store
//    whose other lanes land in a per-wave scratch row, and global memory goes through buffer
//    descriptors whose hardware range check replaces per-lane bounds tests.
//  * Output bits gather in a 64-bit scalar accumulator, flush as big-endian dwords into a VGPR
//    stage and leave as one coalesced 256-byte buffer store per 64 words.
#include <type_traits>

#include "hc_internal.h"

// llvm.amdgcn.writelane has no clang builtin in this toolchain; binding the intrinsic by name
// lets the compiler schedule it and handle its lane-select hazard (unlike inline asm)
extern "C" __device__ int amdgcn_writelane(int x, int l, int v) __asm("llvm.amdgcn.writelane.i32");

namespace hc {

// Test and diagnostic hooks exist only in the debug build (libhcodec_dbg.so, -DHC_DEBUG_HOOKS;
// tests and bench.py's stage pass load it). The shipping libhcodec.so has no mutable globals:
// its windows, tree layouts and encoder modes are the constants below.
#if defined(HC_PROF) && !defined(HC_DEBUG_HOOKS)
#define HC_DEBUG_HOOKS 1
#endif
#ifdef HC_DEBUG_HOOKS
// when non-null, every FGK wave records (start, end, HW_ID | XCC_ID << 16) at [3 * stream]
// (scripts/residency.py measures how many waves share each SIMD); hc_debug_set_trace
__device__ uint64_t *g_trace = nullptr;
// the buffer window (below); hc_debug_set_window shrinks it so that tests cross many window
// edges on small streams
__device__ uint32_t g_window = 1u << 30;
// the lowest tree layout (0 narrow, 1 wide, 2 huge) any stream may use (hc_debug_set_min_tree:
// tests run the wide and huge kernels on small streams); the launchers pass it in Batch::min_tree
static uint32_t g_min_tree = 0;
// encoder mode for narrow / wide streams: 0 = per stream by enc_mode_kernel (default), 1 = path
// cache for all, 2 = tables for all (hc_debug_set_enc_tab; tests run both on every input)
static uint32_t g_enc_tab = 0;
// decoder launch for narrow streams: 0 = by payload rate (dec_small_stream), 1 = small-alphabet
// for all, 2 = regular for all (hc_debug_set_dec_small)
static uint32_t g_dec_small = 0;
__device__ __forceinline__ uint64_t *trace_buf() { return g_trace; }
__device__ __forceinline__ uint32_t window_bytes() { return __builtin_amdgcn_readfirstlane(g_window); }
static uint32_t min_tree() { return g_min_tree; }
static uint32_t enc_tab() { return g_enc_tab; }
static uint32_t dec_small() { return g_dec_small; }
#else
__device__ __forceinline__ uint64_t *trace_buf() { return nullptr; }
__device__ __forceinline__ uint32_t window_bytes() { return 1u << 30; }
static uint32_t min_tree() { return 0; }
static uint32_t enc_tab() { return 0; }
static uint32_t dec_small() { return 0; }
#endif
// Streams are addressed through buffer descriptors, whose offsets are 32-bit: each stream's input
// and output are reached through windows that slide forward by whole multiples of 256 bytes
// once the offset inside them passes window_bytes() (1 GiB), so streams of any length fit.

// the tree layout for a stream of at most `max_sym` FGK symbols
__device__ __forceinline__ uint32_t tree_kind(uint64_t max_sym, uint32_t lo)
{
    const uint32_t k = max_sym <= kNarrowMaxSymbols ? 0u : (max_sym <= kWideMaxSymbols ? 1u : 2u);
    return k > lo ? k : lo;
}

namespace {

__device__ __forceinline__ void trace_wave(uint32_t sid, uint64_t t0, uint32_t lane)
{
    uint64_t *const tr = trace_buf();
#ifdef HC_PROF
    return;  // the buffer holds the path profile (prof_store)
#endif
    if (tr == nullptr) return;
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0) {
        tr[3 * sid] = t0;
        tr[3 * sid + 1] = t1;
        tr[3 * sid + 2] = (hw & 0xFFFFu) | ((xcc & 0xFu) << 16);
    }
}

// Diagnostic build (-DHC_PROF, scripts/path_prof.py): lane i of a per-wave accumulator sums the
// s_memtime cycles spent in region i of the kernel; at the end lanes 0..7 go to g_trace[8 *
// stream + i], lane 0 holding the wave's whole life. Absent from normal builds.
// -DHC_COUNT (with -DHC_PROF): the lanes count events instead (HC_CNT(i): lane i), e.g. the
// batch steps, retests and symbols coded alone of the batched paths
#if defined(HC_PROF) && !defined(HC_COUNT)
#define HC_PROF_BEGIN() const uint64_t hc_p0_ = __builtin_amdgcn_s_memtime()
#define HC_PROF_END(i) (pacc += lane == (i) ? __builtin_amdgcn_s_memtime() - hc_p0_ : 0)
#else
#define HC_PROF_BEGIN()
#define HC_PROF_END(i)
#endif
#ifdef HC_COUNT
#define HC_CNT(i) (pacc += lane == (i) ? 1 : 0)
#else
#define HC_CNT(i)
#endif
__device__ __forceinline__ void prof_store(uint32_t sid, uint64_t t0, uint64_t pacc, uint32_t lane)
{
#ifdef HC_PROF
    uint64_t *const tr = trace_buf();
    if (tr != nullptr && lane < 8) tr[8 * sid + lane] = lane == 0 ? __builtin_amdgcn_s_memtime() - t0 : pacc;
#endif
}

// The issue arbiter prefers higher priority, then older waves: left alone, the oldest of a
// SIMD's 8 waves run ahead and the last ones finish long after, on a half-empty SIMD. Waves
// that are behind (by the share of their stream done: below 1/2, 4/5, 19/20, the rest) take a
// higher priority instead. Within a band the arbiter goes by age, so the last bands are short.
// The band is recomputed only when progress reaches the next band edge (one scalar compare per
// chunk or block; the 64-bit products per call, with their operands spilled, cost ~10 instructions).
template <class I>  // uint32_t, or uint64_t for the huge layout's symbol counts
struct Prio {
    I next = 0;  // the progress at which the band changes next
    __device__ __forceinline__ void at(I done, I total)
    {
        if (done < next) return;
        const uint64_t d = (uint64_t)done * 20, t = total;
        // the band and the first progress past it: ceil(t * k / 20) for k = 10, 16, 19
        uint64_t k;
        if (d < 10 * t) {
            __builtin_amdgcn_s_setprio(3);
            k = 10;
        } else if (d < 16 * t) {
            __builtin_amdgcn_s_setprio(2);
            k = 16;
        } else if (d < 19 * t) {
            __builtin_amdgcn_s_setprio(1);
            k = 19;
        } else {
            __builtin_amdgcn_s_setprio(0);
            k = 0;
        }
        next = k ? (I)((t * k + 19) / 20) : (I)~(I)0;
    }
};

constexpr uint32_t kRoot = 512;
constexpr uint32_t kWords = 576;  // positions 0..512 + sentinels 513..575 (s + 63)
constexpr uint32_t kInner = 0x100;
constexpr uint32_t kNyt = 0x200;
#ifndef HC_WAVES
#define HC_WAVES 4
#endif
constexpr int kWaves = HC_WAVES;  // wavefronts (streams) per workgroup
constexpr uint32_t kMaxBufBytes = 0x7FFFFF00u;  // per-stream limit of the 32-bit buffer offsets
constexpr uint32_t kDrop = 0x7FFFFFF8u;         // buffer offset past every range: access dropped

constexpr uint32_t kMissPos = kWords - 2;  // sentinel: w[kMissPos + 1] <= w[kMissPos], so it fails
constexpr uint32_t kSlots = 16;     // encoder path cache: entries
constexpr uint32_t kSlotDepth = 12; // row capacity: levels per cache entry
#ifndef HC_INSERT_DEPTH
#define HC_INSERT_DEPTH 9
#endif
// deepest path a miss inserts: deeper (rarer) symbols would only evict paths that are used
// again (slot-form model, photo -c -m: misses 5.84 % at 12, 4.95 % at 9, 5.10 % at 8)
constexpr uint32_t kInsertDepth = HC_INSERT_DEPTH;
#ifndef HC_PROBE
#define HC_PROBE 7
#endif
// encoder: a miss chases this many levels, then looks the position reached up in the path cache
constexpr uint32_t kProbe = HC_PROBE;
constexpr uint32_t kRow = 16;       // u16 per cache entry
// 1: path-cache streams (narrow and wide layouts) code cached symbols seven at a time
// (code_all_batch). Code records come from ballots of the positions' parities (C5 encode 433 ->
// 412 ms against reading the cache rows' record words: two LDS operations fewer per step).
// Measured and dropped: uncached symbols joining the batch with lane-parallel chased paths,
// inserted into the cache after the commit (570 ms)
#ifndef HC_ENC_BATCH
#define HC_ENC_BATCH 1
#endif
// decoder (narrow and wide layouts): up to HC_DEC_BATCH (<= 7) codes per step from one read of
// the level tables at every bit offset and one tentative commit (Dec::decode_batch; 0: the
// one-symbol loop only). Measured, C5 decode: one-symbol loop 490 ms, 6 per step 443, 7 per step
// 430; eight per step in 8-lane groups (the root's increments apart) 437; a first code of >= 8
// bits sent to the one-symbol step before the chain (HC_DEC_EXIT8): noise decode 237 -> 198 ms,
// C5 +0.5 %
#ifndef HC_DEC_BATCH
#define HC_DEC_BATCH 7
#endif
#ifndef HC_DEC_EXIT8
#define HC_DEC_EXIT8 1
#endif
// 1: a batch whose first failing symbol's failure may be false (its test counts no earlier batch
// symbol through the next position) is tested again from that symbol with the earlier ones
// committed (code_all_batch, Dec::decode_batch; model: fgk_batch_model.retry_len)
// (measured, grad / C5 / noise, ms: 1 with the plausibility test below, encode 1.50 -> 1.51 / +1 %
// / +0.3 %, decode 1.64 -> 1.66 / +0.7 % / +1 %; 2, the miss test only: encode ±0 / +1.2 % / ±0,
// decode -5.5 % / ±0 / +2 %: the retest's ~35-55 instructions cost what the restarts they save do;
// the decoder's alone, in the blocks of streams that have seen <= 16 symbols (a second copy of the
// block loop): grad decode -2.7 %, C5 decode +0.3 %, C3 decode +0.8 %)
// the encoder vote's spread sample: eight segments' loads in flight at once (enc_mode_kernel)
#ifndef HC_VOTE_BATCH
#define HC_VOTE_BATCH 1
#endif
#ifndef HC_BATCH_RETRY
#define HC_BATCH_RETRY 0
#endif
#ifndef HC_BATCH_YIELD
#define HC_BATCH_YIELD 5
#endif
constexpr uint32_t kBatchYield = HC_BATCH_YIELD;  // Dec::run: twice the symbols per batch worth it
// walk(): after a swap at a position lighter than this, the parent's level is walked at once
// instead of chasing back to the known path. Measured (C5 encode / decode, noise encode /
// decode, ms): never 410 / 397, 206 / 184; always 392 / 381, 218 / 197; below 64: 393 / 381,
// 211 / 190; below 512: 394 / 382, 214 / 193
#ifndef HC_WALK_LIGHT
#define HC_WALK_LIGHT 64
#endif
constexpr uint32_t kWalkLight = HC_WALK_LIGHT;
constexpr uint32_t kSymWords = 88;  // encoder: MNP-5 symbols of one 256-byte chunk, <= 342
                                    // (a byte emits 2 only at a run start that follows a run of
                                    // >= 3, so such bytes are >= 3 apart)
#ifndef HC_REFRESH
#define HC_REFRESH 16
#endif
constexpr uint32_t kRefresh = HC_REFRESH;   // decoder: rebuild the level tables after this many lookups
                                    // they left short of depth 8
constexpr uint32_t kMarkShift = 10; // decoder: body bits 10..14 = table generation (per position)
constexpr uint32_t kNotLeaf = 0x8000; // decoder: body bit 15 = inner or NYT (moves with the content)
constexpr uint32_t kContent = 0x83FF; // decoder: the body bits that move with the content

// Tree layouts by the stream's FGK symbol count (the root's weight): kW = 0 "narrow" (<= 2^22 - 2
// symbols: weight << 10 | parent in one u32), 1 "wide" (< 2^32 - 1: u32 weight, u16 parent), 2
// "huge" (any count: u64 weight, as the reference's uint64_t freq, huffman.hpp:26).
template <int kW>
using WeightT = std::conditional_t<kW == 2, uint64_t, uint32_t>;

// One wavefront's LDS; <= 5 KB so that 8 four-wave workgroups fit a CU (narrow). Encoder and
// decoder each add their cache (tests/fgk_cache_model.py is the executable model of both,
// checked against the plain slot form). kTab: the encoder's table mode (no path cache; the
// decoder's level tables plus pcode[], ~6.5 KB, 6 waves per SIMD).
template <int kW, bool kDec, bool kTab = false, bool kSmall = false>
struct alignas(16) Tree {
    WeightT<kW> wt[kWords];           // narrow: weight << 10 | parent; wide / huge: weight
    uint32_t scratch[kW == 2 ? 128 : 64];  // landing words of lanes that must not write
    // symbol | kInner + child pair | kNyt; decoder: bits 10..15 = generation of the level
    // tables that walked through this position
    uint16_t body[516];
    uint16_t where[kDec ? 2 : 256];   // encoder: symbol -> position | (entry + 1) << 10; 0 = unseen
    uint16_t up[kW ? 516 : 2];        // wide / huge: parent position
    // encoder path cache, entry e = row e: positions of levels 0..11 (kRoot above the path),
    // [12] code record 1 << depth | code bits, [13] depth | valid << 5 | symbol << 8, [14..15]
    // unused. One lane-based
    // address reads a lane's position and (lane 0) the row's metadata.
    // row "entry -1" (where[] entry 0: not cached): level 0 at sentinel position kMissPos, whose
    // leader test always fails at lane 0, so a miss leaves the hot loop like a failed update
    alignas(16) uint16_t pc_miss[(kDec || kTab) ? 2 : kRow];
    uint16_t pc[(kDec || kTab) ? 2 : kSlots * kRow];
    alignas(8) uint32_t syms[kDec ? 64 : kSymWords];  // MNP-5 symbols: encoder one chunk, decoder one block
    // decoder level tables: level j (1..8) at 2^j - 2 + prefix: position | depth << 10 where
    // the walk from the root along the prefix's bits stops; lvl_root (indices -2, -1: "level
    // 0") holds the root, which the lanes above a path's depth read
    uint16_t lvl_root[2];
    uint16_t lvl[(kDec || kTab) ? 512 : 2];
    // table mode: position -> its code as the level tables reached it: the prefix left-aligned
    // to 8 bits | (depth - 1) << 8 (checked against the tables at every use: stale entries fail)
    uint16_t pcode[kTab ? 516 : 2];
    // the small-alphabet kernels (kSmall, narrow layout): the batch steps' membership marks (code_all_batch):
    // bit 16 (a & 1) + j of word (a - 480) >> 1 says batch symbol j's path holds position a (480..513)
    uint32_t smark[kSmall ? 17 : 1];
};

typedef __attribute__((address_space(3))) uint8_t lds_u8;  // a byte in LDS (32-bit address)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
// the 32-bit LDS address of a word of the wave's tree
template <class P>
__device__ __forceinline__ uint32_t lds_off(P *p)
{
    return (uint32_t)(size_t)(__attribute__((address_space(3))) P *)p;
}
__device__ __forceinline__ uint32_t lds_off16(uint16_t *p) { return (uint32_t)(size_t)(lds_u16 *)p; }
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x)
{
    return (uint64_t)uni((uint32_t)x) | ((uint64_t)uni((uint32_t)(x >> 32)) << 32);
}
// the value unchanged, opaque to the optimizer: a u16 LDS load kept as a 32-bit value (left
// alone, masks of it are narrowed to 16-bit ops that cost an extra re-extension each)
__device__ __forceinline__ uint32_t opaque(uint32_t x)
{
    asm("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
// lane l of v := x (x, l wave-uniform): the llvm.amdgcn.writelane intrinsic (declared above)
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t x, uint32_t l)
{
    return (uint32_t)amdgcn_writelane((int)x, (int)l, (int)v);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// lowest set bit of a wave mask, 0xFFFFFFFF for 0 (s_ff1_i32_b64 without the zero test)
__device__ __forceinline__ uint32_t ff1(uint64_t m)
{
    uint32_t r;
    asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
    return r;
}
// the lanes below k: (1 << (k & 63)) - 1 (k = 0xFFFFFFFF: lanes 0..62; in every path vector lane
// 63 holds the root, whose duplicates in the lanes below it store the same word)
__device__ __forceinline__ uint64_t below_mask(uint32_t k)
{
    uint64_t r;
    asm("s_bfm_b64 %0, %1, 0" : "=s"(r) : "s"(k));
    return r;
}
// the lanes of the first j groups of nine, (1 << 9 j) - 1 for j <= 7, on the scalar unit (left to
// itself the compiler may form 9 j on the VALU where SGPRs are scarce)
__device__ __forceinline__ uint64_t groups9(uint32_t j)
{
    uint32_t n;
    uint64_t r;
    asm("s_mul_i32 %0, %1, 9" : "=s"(n) : "s"(j));
    asm("s_bfm_b64 %0, %1, 0" : "=s"(r) : "s"(n));
    return r;
}
// per lane: bit lane of m ? t : f (one v_cndmask on a scalar mask)
__device__ __forceinline__ uint32_t sel(uint64_t m, uint32_t t, uint32_t f)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
// A wave-uniform value held in a VGPR: hiding its uniformity from the compiler moves the
// arithmetic on it from the (saturated) scalar unit to the vector ALUs. Branches on such
// values go through ballot(), which is uniform again.
__device__ __forceinline__ uint32_t vreg(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// lane l gets x of lane l - 1, lane 0 gets fill (a DPP wave shift: no LDS round trip)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t fill)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x138, 0xF, 0xF, false);
}

// Range-checked view of one stream's bytes: base and size, turned into a buffer descriptor at
// each access with readfirstlane on every part. The descriptor must be wave-uniform; kept as a
// value across the loops, the compiler sometimes held it in VGPRs (a u64 min() lowered through
// f64, or SGPR pressure) and wrapped every load through it in a waterfall loop over lanes (~12
// instructions and an exec save per chunk). The readfirstlanes fold away when the parts sit in
// SGPRs, and cost 3 VALU instead of a waterfall when they do not.
struct rsrc_t {
    uint64_t base;
    uint32_t bytes;
};
__device__ __forceinline__ rsrc_t make_rsrc(const uint8_t *p, uint32_t bytes)
{
    return rsrc_t{(uint64_t)(size_t)p, bytes};
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hw_rsrc(rsrc_t r)
{
    // (readfirstlane returns int: each half goes through uint32_t before widening, or a low
    // word with bit 31 set would sign-extend into the high word)
    const uint64_t ua = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r.base) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r.base >> 32)) << 32);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<uint8_t *>((size_t)ua), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(r.bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t buf_load(rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b32(hw_rsrc(r), (int)off, 0, 0);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 buf_load4(rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(hw_rsrc(r), (int)off, 0, 0);
}
__device__ __forceinline__ void buf_store(rsrc_t r, uint32_t off, uint32_t v)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, hw_rsrc(r), (int)off, 0, 0);
}
__device__ __forceinline__ void buf_store8(rsrc_t r, uint32_t off, uint32_t v)
{
    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, hw_rsrc(r), (int)off, 0, 0);
}
__device__ __forceinline__ void buf_store4(rsrc_t r, uint32_t off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, hw_rsrc(r), (int)off, 0, 0);
}

// inclusive prefix sum over the wave (row shifts, then row broadcasts 15 and 31)
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false); // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false); // row_bcast:31
    return x;
}

// ------------------------------------------------------------------------------ the tree --

template <int kW, bool kDec, bool kTab = false, bool kSmall = false>
struct Fgk {
    static constexpr bool kTabs = kDec || kTab;  // keeps the level tables
    static constexpr bool kWide = kW != 0;  // weights apart from parents (wide / huge)
    static constexpr bool kHuge = kW == 2;  // 64-bit weights
    using Wt = WeightT<kW>;
    static constexpr Wt kInc = kWide ? 1u : 1024u;

    Tree<kW, kDec, kTab, kSmall> &T;
    uint32_t lane;
    uint32_t nyt;    // position of the NYT leaf: 512 - 2 * (symbols seen)
    uint32_t bad;    // a structural invariant broke (a bug, never valid input): stop, report
    uint32_t pc_next;  // encoder: FIFO hand of the path cache
    uint32_t pc_free;  // encoder: entries dropped by swaps (or never used), taken first
    uint32_t pc_lb;    // encoder: a weight no cached path's position is below (pc_bound)
    uint32_t pc_lb_ok; // encoder: no insert since pc_bound
    uint32_t gen;      // decoder: generation of the level tables
    uint32_t stale;    // decoder: lookups the level tables left short (kRefresh: from := 0)
    uint32_t from;     // decoder: rebuild levels from..8 of the tables (9: none, 0: all, in a new
                       // generation); a swap moved a position they reach at level from - 1
    const uint16_t *pc_lane;  // encoder: &pc[(lane & 15) - kRow]: where[] entry e's row (0: pc_miss)
    uint64_t pacc = 0;        // HC_PROF regions inside the tree code

    __device__ __forceinline__ Fgk(Tree<kW, kDec, kTab, kSmall> &t, uint32_t l)
        : T(t), lane(l), nyt(kRoot), bad(0), pc_next(0), pc_free(0xFFFFu), pc_lb(0), pc_lb_ok(0), gen(0), stale(0), from(0),
          pc_lane(&t.pc[0] + (l & 15u) - (kTabs ? 0 : kRow))
    {
        // huffman.cpp:23-31: a lone NYT root
        // narrow: sentinels above every weight word; the encoder's last word (above kMissPos)
        // is 0, the decoder's all ones - 1 (see update_fast) but its last 0 too: the pair
        // (kMissPos, kMissPos + 1) fails every leader test
        for (uint32_t i = lane; i < kWords; i += 64)
            T.wt[i] = i <= kRoot ? (Wt)0 : (kWide ? ~(Wt)0 : (Wt)(i == kWords - 1 && (kDec || !kTabs) ? 0u : (kTabs ? 0xFFFFFFFEu : 0xFFFFFFFFu)));
        if (lane < 2) T.lvl_root[lane] = kRoot;
        for (uint32_t i = lane; i < 516; i += 64) {
            T.body[i] = i == kRoot ? (kDec ? kNyt | kNotLeaf : kNyt) : 0;
            if (kWide) T.up[i] = 0;
        }
        if (kSmall && lane < sizeof(T.smark) / 4) T.smark[lane] = 0;
        if (!kDec) {
            for (uint32_t i = lane; i < 256; i += 64) T.where[i] = 0;
            if constexpr (kTab) {
                for (uint32_t i = lane; i < 516; i += 64) T.pcode[i] = 0;
            } else {
                for (uint32_t i = lane; i < kSlots * kRow; i += 64) T.pc[i] = (i % kRow) < kSlotDepth ? 0xFFFF : 0;
                if (lane < kRow) T.pc_miss[lane] = lane == 0 ? kMissPos : kRoot;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }

    // own scratch slot of this lane (16- and 32-bit views)
    __device__ __forceinline__ uint32_t *scr32() const { return &T.scratch[lane]; }
    __device__ __forceinline__ uint16_t *scr16() const
    {
        return reinterpret_cast<uint16_t *>(&T.scratch[lane]);
    }
    __device__ __forceinline__ uint8_t *scr8() const { return reinterpret_cast<uint8_t *>(&T.scratch[lane]); }
    // ... and a weight-sized one
    __device__ __forceinline__ Wt *scrw() const { return reinterpret_cast<Wt *>(&T.scratch[kHuge ? 2 * lane : lane]); }
    // a weight read on the lanes, made wave-uniform / taken from lane l
    static __device__ __forceinline__ Wt uniw(Wt x)
    {
        if constexpr (kHuge) return uni64(x);
        else return uni(x);
    }
    static __device__ __forceinline__ Wt readw(Wt x, uint32_t l)
    {
        if constexpr (kHuge) return (uint64_t)lane_read((uint32_t)x, l) | ((uint64_t)lane_read((uint32_t)(x >> 32), l) << 32);
        else return lane_read(x, l);
    }

    // ---- encoder path cache: root paths of recently coded symbols (tests/fgk_cache_model.py).
    // A path changes only when a swap moves a position on it; splits touch no symbol's path.

    // hit: pr = entry e's row as read lane-parallel at pc_lane[e * kRow] (lane k < 12: position
    // of level k, kRoot padding from the depth on); the path to pv, returns the row's code
    // record (word 12, see RecSink) in an SGPR
    __device__ __forceinline__ uint32_t pc_use(uint32_t e, uint32_t pr, uint32_t &pv)
    {
        pv = lane < kSlotDepth ? pr : kRoot;
        return lane_read(pr, kSlotDepth);
    }

    // forget entry e (its symbol's where[] keeps only the position: level 0 of the path)
    __device__ __forceinline__ void pc_forget(uint32_t e, uint16_t *other, uint32_t oval)
    {
        const uint32_t m = uni(T.pc[e * kRow + kSlotDepth + 1]);
        const uint32_t opos = uni(T.pc[e * kRow]);
        uint16_t *q = lane == 0 ? ((m >> 5) & 1u ? &T.where[m >> 8] : scr16()) : other;
        *q = (uint16_t)(lane == 0 ? opos : oval);
    }

    // after a miss: cache symbol sym at position s with its path (lanes >= d hold kRoot) and
    // its code record rec (1 << d | code bits). Replacement: an entry dropped by a swap (or
    // never used) first, lowest number; otherwise FIFO (tests/fgk_cache_model.py: on the photo
    // streams this misses less than a clock with reference bits, and a hit costs nothing).
    __device__ __forceinline__ void pc_insert(uint32_t sym, uint32_t s, uint32_t pv, uint32_t d, uint32_t rec)
    {
        if (d > kInsertDepth) return;
        pc_lb_ok = 0;
        uint32_t e;
        if (pc_free) {
            e = (uint32_t)__builtin_ctz(pc_free);
            pc_free &= pc_free - 1;
        } else {
            e = pc_next;
            pc_next = (e + 1) & (kSlots - 1);
        }
        // lane 0: the evicted symbol forgets its entry; lane 1: this symbol takes it
        pc_forget(e, lane == 1 ? &T.where[sym] : scr16(), s | ((e + 1) << 10));
        // lanes 0..11 the positions, 12 the code record, 13 depth | valid | symbol
        const uint32_t rv = lane < kSlotDepth ? pv : (lane == kSlotDepth ? rec : (d | 32u | (sym << 8)));
        *(lane < kSlotDepth + 2 ? &T.pc[e * kRow + lane] : scr16()) = (uint16_t)rv;
        __builtin_amdgcn_wave_barrier();
    }

    // pc_lb := the lightest cached leaf. Every position on a cached path weighs at least its
    // leaf and weights only grow, so until the next insert a swap of positions lighter than
    // that (the ties of rare symbols) touches no cached path and needs no scan.
    __device__ __forceinline__ void pc_bound()
    {
        if (pc_lb_ok) return;
        pc_lb_ok = 1;
        if constexpr (kHuge) {  // no bound: every swap scans the cache
            pc_lb = 0;
            return;
        }
        const uint32_t p0 = T.pc[(lane & (kSlots - 1)) * kRow];  // row (lane & 15)'s leaf
        const uint32_t w0 = (uint32_t)T.wt[min(p0, kRoot)];
        uint32_t lw = p0 <= kRoot ? (kWide ? w0 : w0 >> 10) : 0xFFFFFFFFu;  // 0xFFFF: unused row
        lw = min(lw, (uint32_t)__builtin_amdgcn_update_dpp(~0, (int)lw, 0x111, 0xF, 0xF, false));
        lw = min(lw, (uint32_t)__builtin_amdgcn_update_dpp(~0, (int)lw, 0x112, 0xF, 0xF, false));
        lw = min(lw, (uint32_t)__builtin_amdgcn_update_dpp(~0, (int)lw, 0x114, 0xF, 0xF, false));
        lw = min(lw, (uint32_t)__builtin_amdgcn_update_dpp(~0, (int)lw, 0x118, 0xF, 0xF, false));
        pc_lb = lane_read(lw, 15);
    }

    __device__ __forceinline__ void pc_drop(uint32_t e)
    {
        pc_forget(e, scr16(), 0);
        *(lane < kSlotDepth + 2 ? &T.pc[e * kRow + lane] : scr16()) = (uint16_t)(lane < kSlotDepth ? 0xFFFFu : 0u);
        __builtin_amdgcn_wave_barrier();
        pc_free |= 1u << e;
    }

    // positions s and l traded contents: drop every cached path through either. Read r covers
    // entries 4r..4r+3, one position per lane (lane 16j + k: level k of entry 4r + j; words
    // 12..15 of a row are metadata, masked out of the ballot); 16-bit segment j flags entry
    // 4r + j.
    __device__ __forceinline__ void pc_swapped(uint32_t s, uint32_t l)
    {
        constexpr uint64_t kLevels = 0x0FFF0FFF0FFF0FFFull;
        uint32_t q[kSlots / 4];
        uint64_t m[kSlots / 4];
#pragma unroll
        for (uint32_t r = 0; r < kSlots / 4; ++r) q[r] = T.pc[64 * r + lane];
#pragma unroll
        for (uint32_t r = 0; r < kSlots / 4; ++r) m[r] = (ballot(q[r] == s) | ballot(q[r] == l)) & kLevels;
#pragma unroll
        for (uint32_t r = 0; r < kSlots / 4; ++r) {
            while (m[r]) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m[r]) >> 4;
                m[r] &= ~(0xFFFFull << (16 * j));
                pc_drop(4 * r + j);
            }
        }
    }

    // ---- decoder level tables (tests/fgk_cache_model.py: LevelTables). Level j's entry for a
    // j-bit prefix is where the walk from the root along those bits stops (position | depth <<
    // 10); built breadth first, each level from the one above. A swap stales them only when it
    // moves the content of a position some walk passes through: those carry the generation.
    // from = 0: all levels, a new generation; otherwise levels from..8 (the entries above reach
    // neither swapped position, so they and the marks they set stand)
    __device__ __forceinline__ void build_levels()
    {
        uint32_t j0 = from;
        if (j0 == 0) {
            gen = gen == 31 ? 1u : gen + 1;
            j0 = 1;
            stale = 0;
        }
        from = 9;
#pragma unroll 1
        for (uint32_t j = j0; j <= 8; ++j) {
            const uint32_t cnt = 1u << j;
            for (uint32_t r = 0; r * 64 < cnt; ++r) {
                const uint32_t q = lane + 64 * r;
                const bool on = q < cnt;
                const uint32_t pe = j == 1 ? kRoot : T.lvl[(cnt >> 1) - 2 + (on ? q >> 1 : 0)];
                const uint32_t x = pe & 1023u;
                const uint32_t b = T.body[x];
                const bool inner = (b & kInner) && (pe >> 10) == j - 1;
                *(on && inner ? &T.body[x] : scr16()) = (uint16_t)((b & kContent) | (gen << kMarkShift));
                const uint32_t ne = inner ? (((b & 255u) * 2 + (q & 1u)) | (j << 10)) : pe;
                *(on ? &T.lvl[cnt - 2 + q] : scr16()) = (uint16_t)ne;
                if constexpr (kTab)  // the child reached at depth j has code q
                    *(on && inner ? &T.pcode[(b & 255u) * 2 + (q & 1u)] : scr16()) = (uint16_t)((q << (8 - j)) | ((j - 1) << 8));
            }
            __builtin_amdgcn_wave_barrier();
        }
    }

    // decoder: the shallowest level < 8 whose entries hold position s or l (8 if none does).
    // Level j's entries sit at 2^j - 2 .. 2^(j+1) - 3 and a position first appears at its
    // depth, so the lowest matching index names it (level 8's entries stay right: a position
    // they stop at is walked on by the descent). Entries of levels >= from may predate a swap
    // earlier in this walk; a match there gives a level >= from - 1, leaving from as it is.
    __device__ __forceinline__ uint32_t table_level(uint32_t s, uint32_t l)
    {
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t i = r * 64 + lane;
            const uint32_t p = T.lvl[i] & 1023u;
            const uint64_t m = (ballot(p == s) | ballot(p == l)) & (r == 3 ? 0x3FFFFFFFFFFFFFFFull : ~0ull);
            if (m) return 31 - __builtin_clz(r * 64 + ff1(m) + 2);
        }
        return 8;
    }

    // huffman.cpp:99-111: split NYT at t -> NYT at t-2 (left), symbol leaf at t-1 (right).
    // Lanes 0..2 write the three bodies, lanes 0..1 the two parent links, lane 0 the map.
    __device__ __forceinline__ uint32_t split(uint32_t sym)
    {
        const uint32_t t = nyt;
        const uint32_t bpos = lane == 0 ? t : (lane == 1 ? t - 2 : t - 1);
        constexpr uint32_t nl = kDec ? kNotLeaf : 0u;
        const uint32_t bval = lane == 0 ? (kInner | nl | ((t - 2) >> 1)) : (lane == 1 ? kNyt | nl : sym);
        *(lane < 3 ? &T.body[bpos] : scr16()) = (uint16_t)bval;
        if (!kDec) *(lane == 0 ? &T.where[sym] : scr16()) = (uint16_t)(t - 1);
        if constexpr (kWide) *(lane < 2 ? &T.up[t - 2 + lane] : scr16()) = (uint16_t)t;
        else *(lane < 2 ? &T.wt[t - 2 + lane] : scr32()) = t;  // weight 0, parent t
        __builtin_amdgcn_wave_barrier();
        nyt = t - 2;
        return t - 1;
    }

    // huffman.cpp:186-217 in slot form: exchange the contents of positions s and l (their
    // weights are equal), then re-point what hangs below them. Lane k < 2 writes the content
    // moving into (k ? l : s); lane k < 4 re-parents child (k & 1) of content (k >> 1).
    __device__ __forceinline__ void swap(uint32_t s, uint32_t l, bool scan)
    {
        // encoder: drop the cached paths through s or l first (scan: they may lie on one); the
        // relink below then gives a moved leaf's where[] its new position
        if (!kTabs && scan) {
            HC_PROF_BEGIN();
            pc_swapped(s, l);
            HC_PROF_END(7);
        }
        // lane-parallel: lane & 1 = 0 handles the content moving to s (read at l), 1 the one
        // moving to l; lanes 2, 3 (lane >> 1 = 1) re-parent the second child of the same content
        const uint32_t pos = (lane & 1) ? l : s;        // where the lane's content goes
        const uint32_t b = T.body[(lane & 1) ? s : l];  // that content
        if (kTabs) {
            // generation marks stay with the positions: the destination's own word is the
            // partner lane's read (quad_perm [1,0,3,2])
            const uint32_t bo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false);
            *(lane < 2 ? &T.body[pos] : scr16()) = (uint16_t)((b & kContent) | (bo & (31u << kMarkShift)));
            if (ballot(((b >> kMarkShift) & 31u) == gen) & 3u) from = min(from, table_level(s, l) + 1);
            if (!kDec) *(lane < 2 && !(b & kInner) ? &T.where[b & 255u] : scr16()) = (uint16_t)pos;
        } else {
            *(lane < 2 ? &T.body[pos] : scr16()) = (uint16_t)b;
            *(lane < 2 && !(b & kInner) ? &T.where[b & 255u] : scr16()) = (uint16_t)pos;
        }
        const bool inner = lane < 4 && (b & kInner);
        const uint32_t c = (b & 255u) * 2 + (lane >> 1);
        if constexpr (kWide) {
            *(inner ? &T.up[c] : scr16()) = (uint16_t)pos;
        } else {
            // the parent field, in place: LDS and / or without return (no read round trip; this
            // wave's later LDS reads come after them in order)
            uint32_t *q = inner ? &T.wt[c] : scr32();
            __hip_atomic_fetch_and(q, ~1023u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_or(q, pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        __builtin_amdgcn_wave_barrier();
    }

    // highest position >= from whose weight equals that of word w, when positions
    // from-64..from-1 all had it (the sentinels above the root end the scan)
    __device__ __forceinline__ uint32_t leader_far(uint32_t from, Wt w)
    {
        const Wt lim = kWide ? w : (w | 1023u);
        for (;;) {
            const uint64_t le = ballot(T.wt[min(from + lane, kWords - 1)] <= lim);
            if (le != ~0ull) return from + (uint32_t)__builtin_ctzll(~le) - 1;
            from += 64;
        }
    }

    // decoder: the position of symbol sym's leaf, 0xFFFFFFFF if it has none (lane-parallel scan
    // of body[]; only a corrupted stream names a known symbol after the NYT code)
    __device__ __forceinline__ uint32_t find_leaf(uint32_t sym)
    {
        for (uint32_t r = 0; r * 64 <= kRoot; ++r) {
            const uint32_t p = r * 64 + lane;
            const uint32_t b = T.body[min(p, kRoot)];
            // positions at or below the NYT are unused (body 0 would read as symbol 0)
            const uint64_t m = ballot(p > nyt && p <= kRoot && !(b & (kInner | kNyt)) && (b & 255u) == sym);
            if (m) return r * 64 + (uint32_t)__builtin_ctzll(m);
        }
        return 0xFFFFFFFFu;
    }

    __device__ __forceinline__ uint32_t parent(uint32_t x) const
    {
        return kWide ? uni(T.up[x]) : (uni((uint32_t)T.wt[x]) & 1023u);
    }

    // Encoder: the path from position s to the root, BEFORE the update (the code of
    // huffman.cpp:136-155): the position of level k (0 = s) goes to lane k; returns the levels.
    // Each level enters at lane 0 by a DPP wave shift (lane 0 keeps the new position), so the
    // path arrives top-down; one permute turns it bottom-up at the end.
    __device__ __forceinline__ uint32_t chase(uint32_t s0, uint32_t &pv)
    {
        int32_t km = -64;       // levels - 64
        uint32_t s = vreg(s0);  // per-level work on the VALU (see vreg)
        uint32_t td = kRoot;    // lane j: level k - 1 - j
        if (!kTabs) {
            // encoder: kProbe levels, then look the position up in the path cache: a cached
            // path through it (rows stay valid paths) gives the rest of the climb at once
#pragma unroll
            for (uint32_t i = 0; i < kProbe; ++i) {
                const uint32_t sh = __builtin_amdgcn_update_dpp(0u, td, 0x138, 0xF, 0xF, true);
                td = lane == 0 ? s : sh;
                ++km;
                s = kWide ? (uint32_t)T.up[s] : ((uint32_t)T.wt[s] & 1023u);
                if (uni(s) == kRoot) break;
            }
            const uint32_t c = uni(s);
            if (c != kRoot) {
                constexpr uint64_t kLevels = 0x0FFF0FFF0FFF0FFFull;
                uint32_t q[kSlots / 4];
                uint64_t m[kSlots / 4];
#pragma unroll
                for (uint32_t r = 0; r < kSlots / 4; ++r) q[r] = T.pc[64 * r + lane];
#pragma unroll
                for (uint32_t r = 0; r < kSlots / 4; ++r) m[r] = ballot(q[r] == c) & kLevels;
                const uint64_t m01 = m[0] | m[1], m23 = m[2] | m[3];
                if (m01 | m23) {
                    // the first hit: entry e, level lv of its row
                    const uint32_t r = m01 ? (m[0] ? 0u : 1u) : (m[2] ? 2u : 3u);
                    const uint32_t b = ff1(r == 0 ? m[0] : r == 1 ? m[1] : r == 2 ? m[2] : m[3]);
                    const uint32_t e = 4 * r + (b >> 4), lv = b & 15u;
                    const uint32_t n = (uint32_t)(km + 64);  // levels chased: c is level n
                    // lane j >= n: level j = the row's level lv + j - n (kRoot from the row's
                    // depth on, and past its 12 levels)
                    const uint32_t idx = lv + lane - n;
                    const uint32_t rv = T.pc[e * kRow + min(idx, kRow - 1)];
                    const uint32_t drow = uni(T.pc[e * kRow + kSlotDepth + 1]) & 31u;
                    const uint32_t dn =
                        (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((n - 1 - lane) & 63u) * 4), (int)td);
                    pv = lane < n ? dn : (idx < kSlotDepth ? rv : kRoot);
                    return n + drow - lv;
                }
            }
        }
        if (kTabs || uni(s) != kRoot) do {
            // wave_shr:1, lane 0 taking s
            const uint32_t sh = __builtin_amdgcn_update_dpp(0u, td, 0x138, 0xF, 0xF, true);
            td = lane == 0 ? s : sh;
            ++km;
            s = kWide ? (uint32_t)T.up[s] : ((uint32_t)T.wt[s] & 1023u);
            // go on while s is not the root (x - 1 >= 0) and fewer than 64 levels (km < 0;
            // parents sit above children, so this only bounds a bug): one sign test
        } while ((int32_t)((uint32_t)km & ~((uni(s) ^ kRoot) - 1u)) < 0);
        uint32_t k = (uint32_t)(km + 64);
        asm volatile("" : "+s"(k));  // the depth, opaque: no loop-strength-reduced copies of it
        bad |= uni(s) ^ kRoot;
        const uint32_t j = k - 1 - lane;  // lane < k: the lane holding this lane's level
        pv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((j & 63u) * 4), (int)td);
        pv = lane < k ? pv : kRoot;
        return k;
    }

    // huffman.cpp:95-128 (update), serial form, from position s upward: per level one
    // lane-parallel read of positions s..s+63, one ballot (the trailing-ones count of
    // "weight == w[s]" is the block leader, highest number first), a swap when the leader is
    // neither s nor its parent, one store.
    // pv: the root path the update started on (lane k: level k, kRoot lanes above). After the
    // level at s, the climb from its parent is chased (one LDS read per position, no leader
    // test) until it meets a position of pv -- every swap so far moved only positions below
    // that one, and pv's kRoot lanes end any climb at the root. The chased positions and pv
    // above the meeting point are the rest of the root path, finished lane-parallel like
    // update_fast; a level that reports there is walked again, the new path taking pv's role.
    // bounded: the encoder's pc_lb is current (pc_bound since the last insert): swaps below it
    // skip the cache scan
    __device__ __forceinline__ void walk(uint32_t s, uint32_t pv, bool bounded = false)
    {
        for (;;) {
            const Wt v = T.wt[s + lane];  // sentinels cover s + 63 <= 575
            Wt ws = uniw(v);
            const uint64_t le = ballot(v <= (kWide ? ws : (ws | 1023u)));
            uint32_t p = kWide ? uni(T.up[s]) : ((uint32_t)ws & 1023u);
            // lane 0 read position s: its address and word, incremented, are the store's
            Wt *dst = &T.wt[s + lane];
            Wt nv = v + kInc;
            bool again = false;  // the parent's level is walked too (no chase)
            if ((uint32_t)le & 2u) {  // s+1 weighs the same: find the block leader
                const uint32_t lead =
                    ~le ? s + (uint32_t)__builtin_ctzll(~le) - 1 : leader_far(s + 64, ws);
                if (lead != p) {
                    // a light position that swapped: in the long blocks of equal small weights
                    // its new parent usually ties as well, and testing it here costs one read
                    // where the chase back to pv and update_from cost several
                    again = (kWide ? ws : ws >> 10) < kWalkLight;
                    swap(s, lead, !kDec && (!bounded || (kWide ? ws : ws >> 10) >= pc_lb));
                    // the swap rewrites only parent fields below s and lead, never their own
                    // words, so the pre-swap read still holds lead's word when in range
                    const uint32_t off = lead - s;
                    ws = off < 64 ? readw(v, off) : uniw(T.wt[lead]);
                    s = lead;
                    p = kWide ? uni(T.up[s]) : ((uint32_t)ws & 1023u);
                    dst = &T.wt[s];
                    nv = ws + kInc;
                }
            }
            *(lane == 0 ? dst : scrw()) = nv;
            __builtin_amdgcn_wave_barrier();
            if (again && p != kRoot) {
                s = p;
                continue;
            }
            // chase from the parent until a position of pv; lane j of td: the j-th one passed. The
            // climbing position stays in a VGPR (wave-uniform): each level is a compare, a select
            // into lane n (a scalar bit mask), the parent read and a mask -- no hop through the
            // scalar unit (with the position in an SGPR the compiler spent ~6 VALU + 11 SALU per
            // level on copies, readfirstlane and the address)
            uint32_t c = vreg(p), n = 0, td = kRoot;
            uint64_t on;
#pragma unroll 1
            while ((on = ballot(pv == c)) == 0) {
                td = sel(1ull << n, c, td);
                if (++n >= 63) {  // a valid path is shorter (pv's kRoot lanes end every climb): a bug
                    bad = 1;
                    return;
                }
                c = kWide ? (uint32_t)T.up[c] : ((uint32_t)T.wt[c] & 1023u);
            }
            // lane j < n: chased; lane j >= n: pv's lane j - n + m (kRoot past its lane 63)
            const uint32_t src = lane - n + ff1(on);
            const uint32_t up = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src * 4), (int)pv);
            pv = lane < n ? td : (src < 64 ? up : kRoot);
            const uint32_t k = update_from(pv, 0);
            if (k == 0xFFFFFFFFu) return;  // the root too
            s = lane_read(pv, k);
        }
    }

    // The same update when the path is already known: lanes 0..d-1 hold the positions of
    // levels 0..d-1, the other lanes kRoot. Until the first swap the tree does not change, so
    // every level's leader test reads the pre-update words in parallel. A level leads its block
    // when the next position is heavier; the test cannot miss a non-leader, and it reports one
    // falsely only when that next position is the level's own parent and the sibling weighs 0
    // (the NYT): the walk, which repeats the exact test from the first reported level, handles
    // both. The root lanes always lead (the sentinel above is heavier). Levels below the first
    // reported one increment with one store; without a report the root lanes bump the root in
    // the same store. update_fast() is this lane-parallel part; it returns the first reported
    // level (0xFFFFFFFF: none), where walk() continues.
    // force (wave-uniform, 0 or 0xFFFFFFFF): report level 0, store nothing (the limit becomes
    // all ones, above every weight word and sentinel)
    template <class Ahead>
    __device__ __forceinline__ uint32_t update_fast(uint32_t a, Ahead &&ahead, uint32_t force = 0)
    {
        const Wt w0 = T.wt[a], w1 = T.wt[a + 1];
        ahead();  // the caller's reads for later symbols go out behind these
        const Wt nv = w0 + kInc;
        const Wt fw = (Wt)0 - (Wt)(force & 1u);  // force as a weight-wide mask
        // narrow: w1 < w0 + 1024 (the increment stored anyway) reports every level whose next
        // position is not heavier, and falsely (the walk then decides) only one whose next
        // position is exactly one heavier with a lower parent field (parents grow with the
        // position in practice: 0 of 600k level tests on a photo stream, 1 of 7.7k on a
        // gradient, slot-form model). The encoder's miss row's sentinel pair (all ones, 0)
        // fails: all ones + 1024 wraps to 1023; the decoder's force makes the limit all ones,
        // above its sentinels (all ones - 1).
        const uint64_t fail = ballot(kHuge ? (w1 <= (w0 | fw)) : kWide ? (w1 <= (w0 | force | (force >> 1))) : (w1 < (nv | force)));
        const uint32_t k = ff1(fail);  // 0xFFFFFFFF without a failure: every lane increments
        // lanes below k store: the select runs on a scalar mask (s_bfm_b64), one vector op
        // (measured: an exec-masked store, s_bfm + save/restore of exec, made the encoder 3 %
        // slower than a compare and select)
        *(__attribute__((address_space(3))) Wt *)(size_t)sel(below_mask(k), lds_off(&T.wt[a]), lds_off(scrw())) = nv;
        __builtin_amdgcn_wave_barrier();
        return k;
    }
    // update_fast for the levels from lane m up (the lanes below are levels already done):
    // returns the first reported level >= m (0xFFFFFFFF: none, the root lanes bumped the root)
    __device__ __forceinline__ uint32_t update_from(uint32_t a, uint32_t m)
    {
        const Wt w0 = T.wt[a], w1 = T.wt[a + 1];
        const Wt nv = w0 + kInc;
        const uint64_t lo = below_mask(m);
        const uint64_t fail = ballot(kWide ? (w1 <= w0) : (w1 < nv)) & ~lo;
        const uint32_t k = ff1(fail);
        *(__attribute__((address_space(3))) Wt *)(size_t)sel(below_mask(k) & ~lo, lds_off(&T.wt[a]), lds_off(scrw())) = nv;
        __builtin_amdgcn_wave_barrier();
        return k;
    }
    __device__ __forceinline__ void update_path(uint32_t a)
    {
        const uint32_t k = update_fast(a, [] {});
        if (k != 0xFFFFFFFFu) walk(lane_read(a, k), a);
    }
};

// -------------------------------------------------------------- MNP-5 pre-pass (encoder) --

// Carry between chunks: last raw byte (diff model), run counter after the last byte (0 = no
// run: stream start or a 258-byte cut), last transformed byte.
struct RleCarry {
    uint32_t x, R, c;
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, uint32_t b) { return (w >> (8 * b)) & 255u; }

// transform.cpp:220-229 + 241-279 for one chunk, all lanes at once (model and derivation:
// tests/rle_chunk_model.py). Lane l holds raw bytes 4l..4l+3 of the chunk in x4, m (1..256) are
// valid, fin says byte m-1 is the stream's last. Per byte: k = offset in its run (the run may
// continue from the previous chunk), km = k mod 258, run counter R = km + 1 (0 at the cut);
// a byte emits the previous run's count byte and itself when a run starts (or it is the final
// byte), itself at km 1..2, 255 at km 257, nothing otherwise. The chunk's symbols are appended
// to the at symbols pending in sb[] (room for cap); returns the symbols pending after the chunk,
// or -- when they would not fit -- sets full, writes nothing and leaves the carry as it was (the
// caller codes the pending symbols and runs the chunk again).
// Fast path (rle_chunk_model.pure_chunk): a full, non-final chunk whose 256 transformed bytes all
// continue the carried byte's run puts byte i at km = (R + i) mod 258, so it emits only the
// events of the residues 257 (255), 0, 1, 2 (the byte) that fall on i <= 255: in byte order the
// cyclic order 257, 0, 1, 2 rotated to start at R when R <= 2, lane j < 4 taking entry j.
template <int kSrc>
__device__ __forceinline__ uint32_t rle_chunk(uint32_t x4, uint32_t m, uint32_t fin, RleCarry &cy, uint8_t *sb,
                                              uint32_t at, uint32_t cap, uint32_t *scr, uint32_t lane, uint32_t &full,
                                              uint32_t &start_lanes)
{
    const uint32_t xprev = (x4 << 8) | (wave_shr1(x4, cy.x << 24) >> 24);
    // bytewise x - xprev (mod 256), SWAR
    const uint32_t c4 = kSrc == SRC_RAW_DIFF
                            ? (((x4 | 0x80808080u) - (xprev & 0x7F7F7F7Fu)) ^ ((x4 ^ ~xprev) & 0x80808080u))
                            : x4;
    uint8_t *sc = reinterpret_cast<uint8_t *>(scr);
    if (m == 256 && !fin && ballot(c4 != cy.c * 0x01010101u) == 0) {
        start_lanes = cy.R == 0 ? 1u : 0u;
        const uint32_t R = cy.R;
        const uint32_t rot = R <= 2 ? R + 1 : 0;
        const uint32_t q = (lane + rot) & 3u;
        const uint32_t e = q == 0 ? 257u : q - 1;
        uint32_t i = e + 258 - R;
        i = i >= 258 ? i - 258 : i;
        const bool on = lane < 4 && i <= 255;
        const uint32_t total = (uint32_t)__builtin_popcountll(ballot(on));
        if (at + total > cap) {
            full = 1;
            return at;
        }
        *(on ? sb + at + lane : sc) = (uint8_t)(e == 257 ? 255u : cy.c);
        __builtin_amdgcn_wave_barrier();
        cy.x = lane_read(x4, 63) >> 24;
        cy.R = R + 256 >= 258 ? R - 2 : R + 256;
        return at + total;
    }
    const uint32_t cprev = (c4 << 8) | (wave_shr1(c4, cy.c << 24) >> 24);
    const int i0 = (int)(lane * 4);
    uint32_t start[4], any = 0;
    int last = -1;
    for (uint32_t b = 0; b < 4; ++b) {
        uint32_t same = byte_of(c4, b) == byte_of(cprev, b);
        if (b == 0) same &= lane != 0 || cy.R != 0;  // lane 0 byte 0: continues the carry's run?
        start[b] = (uint32_t)(i0 + (int)b < (int)m) & (same ^ 1u);
        any |= start[b];
        last = start[b] ? i0 + (int)b : last;
    }
    // latest run start in the lanes below (else the carried run, begun at -R)
    const uint64_t anyl = ballot(any != 0);
    start_lanes = (uint32_t)__builtin_popcountll(anyl);
    const uint64_t amask = anyl & ((1ull << lane) - 1ull);
    const int src = amask ? 63 - __builtin_clzll(amask) : 0;
    const int below = __builtin_amdgcn_ds_bpermute(src * 4, last);
    int ls = amask ? below : -(int)cy.R;
    uint32_t R[4], km[4];
    for (uint32_t b = 0; b < 4; ++b) {
        ls = start[b] ? i0 + (int)b : ls;
        const uint32_t k = (uint32_t)(i0 + (int)b - ls);
        km[b] = k >= 258 ? k - 258 : k;
        R[b] = km[b] == 257 ? 0u : km[b] + 1;
    }
    const uint32_t upR = wave_shr1(R[3], cy.R);
    uint32_t n[4], s0[4], s1[4], tot = 0;
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t i = (uint32_t)i0 + b;
        const uint32_t rp = b ? R[b - 1] : upR;
        const uint32_t c = byte_of(c4, b);
        const uint32_t valid = i < m ? 1u : 0u;
        const uint32_t newrun = ((fin & (i + 1 == m ? 1u : 0u)) | (km[b] == 0 ? 1u : 0u));
        const uint32_t cnt = newrun & (rp >= 3 ? 1u : 0u);
        const uint32_t lit = km[b] == 1 || km[b] == 2 ? 1u : 0u;
        const uint32_t cut = km[b] == 257 && !newrun ? 1u : 0u;
        n[b] = valid * (newrun ? 1 + cnt : (lit | cut));
        s0[b] = cnt ? rp - 3 : (cut ? 255u : c);
        s1[b] = c;
        tot += n[b];
    }
    // exclusive prefix of the per-lane totals (<= 8): bit planes, ballot + mbcnt
    uint32_t basepos = 0;
    for (uint32_t p = 0; p < 4; ++p) {
        const uint64_t bm = ballot((tot >> p) & 1u);
        basepos += __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << p;
    }
    const uint32_t total = lane_read(basepos + tot, 63);
    if (at + total > cap) {
        full = 1;
        return at;
    }
    uint32_t o = at + basepos;
    for (uint32_t b = 0; b < 4; ++b) {
        *(n[b] >= 1 ? sb + o : sc) = (uint8_t)s0[b];
        *(n[b] == 2 ? sb + o + 1 : sc + 1) = (uint8_t)s1[b];
        o += n[b];
    }
    __builtin_amdgcn_wave_barrier();
    // carries: the chunk's last byte
    const uint32_t L = m - 1, ll = L >> 2, lb = L & 3u;
    const uint32_t rl = lb == 0 ? R[0] : (lb == 1 ? R[1] : (lb == 2 ? R[2] : R[3]));
    cy.x = byte_of(lane_read(x4, ll), lb);
    cy.c = byte_of(lane_read(c4, ll), lb);
    cy.R = lane_read(rl, ll);
    return at + total;
}

// A full, non-final block of kQ KB of a run-heavy stream (tests/rle_chunk_model.py: sparse_block,
// rle_blocked), lane l holding bytes 16 kQ l .. 16 kQ l + 16 kQ - 1 in x[0..4 kQ) (kQ 16-byte
// loads). When the block has at most kSparseStarts run starts and at most 63 symbols, it is coded
// by segments instead of byte by byte: the carried segment [0, p_0) continues the run before the
// block, and segment j = [p_j, p_j+1) is a new run. A segment emits its start's count (when the
// run before it reached R' >= 3: R' - 3) and c, then a symbol for every offset whose residue mod
// 258 is 0, 1, 2 (c) or 257 (255): the t-th of those is 255 when t % 4 == 3. The carried segment's
// residues start at the carried counter R instead. Lane j < S holds start j (its segment's length
// and event count), a scan of the counts places the segments, and each symbol's lane finds its
// segment by a max-scan over markers (one LDS row). Returns the symbols pending after the block,
// or kDense with nothing written and the carry unchanged (the caller then codes the block as
// 256-byte chunks). The caller guarantees room for 63 symbols.
#ifndef HC_SPARSE
#define HC_SPARSE 1
#endif
// KB per sparse block (1 or 2): 2 halves the blocks of a run-heavy stream (grad: every 2 KB block
// stays within the 16 starts and 63 symbols, slot-form model), 4 KB would not fit them
#ifndef HC_SPARSE_KB
#define HC_SPARSE_KB 2
#endif
// rle_block's start mask is 32 bits (one per run start slot), its positions stay below 2048 and
// mod258's exactness bound (v < 2321) holds only up to 2 KB blocks
static_assert(HC_SPARSE_KB == 1 || HC_SPARSE_KB == 2, "rle_block supports 1 KB and 2 KB sparse blocks only");
constexpr uint32_t kSparseStarts = 16;
constexpr uint32_t kDense = 0xFFFFFFFFu;
template <int kSrc, uint32_t kQ>
__device__ __forceinline__ uint32_t rle_block(const u32x4 *blk, RleCarry &cy, uint8_t *sb, uint32_t at, uint32_t *row,
                                              uint32_t lane)
{
    constexpr uint32_t kX = 4 * kQ;          // dwords per lane
    constexpr uint32_t kBytes = 1024 * kQ;   // bytes per block
    uint32_t x[kX];
#pragma unroll
    for (uint32_t k = 0; k < kX; ++k) x[k] = blk[k >> 2][k & 3];
    // transform.cpp:220-229: the diffed bytes (lane 0's previous byte is the carry's)
    uint32_t c[kX];
    uint32_t pb = wave_shr1(x[kX - 1], cy.x << 24) >> 24;
#pragma unroll
    for (uint32_t k = 0; k < kX; ++k) {
        const uint32_t xp = (x[k] << 8) | pb;
        c[k] = kSrc == SRC_RAW_DIFF ? (((x[k] | 0x80808080u) - (xp & 0x7F7F7F7Fu)) ^ ((x[k] ^ ~xp) & 0x80808080u)) : x[k];
        pb = x[k] >> 24;
    }
    // run starts: bit 4 k + b of M for byte b of c[k] (byte 0 of the block also when R = 0: a cut)
    uint32_t M = 0;
    pb = wave_shr1(c[kX - 1], cy.c << 24) >> 24;
#pragma unroll
    for (uint32_t k = 0; k < kX; ++k) {
        const uint32_t d = c[k] ^ ((c[k] << 8) | pb);
        const uint32_t f = ((((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u) >> 7;  // 1 per nonzero byte
        M |= ((f | (f >> 7) | (f >> 14) | (f >> 21)) & 15u) << (4 * k);
        pb = c[k] >> 24;
    }
    M |= lane == 0 && cy.R == 0 ? 1u : 0u;
    const uint32_t cnt = (uint32_t)__builtin_popcount(M);
    const uint32_t incl = wave_scan_add(cnt);
    const uint32_t S = lane_read(incl, 63);
    if (S > kSparseStarts) return kDense;
    // the starts in order: row[r] = position | run byte << 16 (writes past S land on row[63])
    {
        uint32_t r = incl - cnt, m = M;
        while (ballot(m != 0)) {
            const uint32_t b = m ? (uint32_t)__builtin_ctz(m) : 0u;
            uint32_t ck = c[0];
#pragma unroll
            for (uint32_t k = 1; k < kX; ++k) ck = (b >> 2) == k ? c[k] : ck;
            row[m ? r : 63u] = (lane * 4 * kX + b) | (((ck >> (8 * (b & 3u))) & 255u) << 16);
            r += m ? 1u : 0u;
            m &= m - 1u;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t pw = row[lane];
    const bool st = lane < S;
    const uint32_t p = st ? pw & 0xFFFFu : kBytes;
    const uint32_t cb = (pw >> 16) & 255u;
    const uint32_t R0 = cy.R;
    const uint32_t p0 = S ? lane_read(p, 0) : kBytes;
    // segment j: [p, pn); the run counter before its start: (R0 + p_0) mod 258 for j = 0, the
    // previous new run's length mod 258 otherwise
    const uint32_t pn = (uint32_t)__builtin_amdgcn_update_dpp((int)kBytes, (int)p, 0x130, 0xF, 0xF, false);  // wave_shl:1
    const uint32_t pp = wave_shr1(p, 0u);
    const uint32_t L = pn - p;
    auto mod258 = [](uint32_t v) {  // v < 2321 (the largest here: R0 + 2048 < 2306)
        return v - 258u * ((v * 2033u) >> 19);
    };
    const uint32_t Rp = mod258(lane == 0 ? R0 + p : p - pp);
    const uint32_t hc = Rp >= 3 ? 1u : 0u;  // the start emits a count R' - 3 first
    const uint32_t qL = (L * 2033u) >> 19;
    const uint32_t ne = st ? hc + 4 * qL + min(L - 258u * qL, 3u) : 0u;
    const uint32_t ninc = wave_scan_add(ne);
    // the carried segment: lane t < 16 kQ tests its t-th candidate (cycle t >> 2, entry t & 3 of
    // 257, 0, 1, 2 rotated to start at R0)
    const uint32_t rot = R0 <= 2 ? R0 + 1 : 0u;
    const uint32_t q = (lane + rot) & 3u;
    const uint32_t e = q == 0 ? 257u : q - 1u;
    const uint32_t ic = mod258(e + 258u - R0) + 258u * (lane >> 2);
    const uint32_t nc = (uint32_t)__builtin_popcountll(ballot(lane < 16 * kQ && ic < p0));
    const uint32_t total = nc + lane_read(ninc, 63);
    if (total > 63) return kDense;
    // markers: each start's key (its first symbol's index, count flag and value, run byte) at row
    // [its index]; an inclusive max-scan gives every symbol lane its segment (0: the carried one)
    row[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    const uint32_t base = nc + ninc - ne;
    row[st ? base : 63u] = 0x80000000u | (base << 24) | (hc << 23) | (((Rp - 3u) & 255u) << 8) | cb;
    __builtin_amdgcn_wave_barrier();
    uint32_t key = row[lane];
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x111, 0xF, 0xF, false));  // row_shr:1
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x112, 0xF, 0xF, false));  // row_shr:2
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x114, 0xF, 0xF, false));  // row_shr:4
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x118, 0xF, 0xF, false));  // row_shr:8
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x142, 0xA, 0xF, false));  // row_bcast:15
    key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x143, 0xC, 0xF, false));  // row_bcast:31
    // a start segment's symbol (selects per lane), else the carried segment's
    const uint32_t u = lane - ((key >> 24) & 63u), kc = (key >> 23) & 1u;
    const uint32_t vs = kc && u == 0 ? (key >> 8) & 255u : (((u - kc) & 3u) == 3u ? 255u : key & 255u);
    const uint32_t v = (key >> 31) ? vs : (e == 257 ? 255u : cy.c);
    *(lane < total ? sb + at + lane : reinterpret_cast<uint8_t *>(row + 63)) = (uint8_t)v;
    __builtin_amdgcn_wave_barrier();
    // carries: the block's last raw and diffed byte, the run counter after it
    cy.x = lane_read(x[kX - 1], 63) >> 24;
    cy.c = lane_read(c[kX - 1], 63) >> 24;
    cy.R = mod258(S ? kBytes - lane_read(p, S - 1) : R0 + kBytes);
    return at + total;
}

// ------------------------------------------------------------------------- output stage --

// Code records: the encoder does not shift bits per symbol. Symbol t's code becomes one record
// in lane t of a VGPR, 1 << len | code (len <= 31; the leading 1 marks the length), written with
// one compare + select. Every 64 records (and at the end) pack() turns them into bytes on the
// lanes: a DPP scan of the lengths gives each record its bit offset, each record ORs its head
// (and the tail that spills into the next word) into a 64-word LDS stage, and the complete
// words leave as one buffer store, big-endian. 64 records of <= 31 bits plus < 32 pending bits
// fill at most 63 words. The u64 count (words 0-1) is written at the end by the lanes that
// stored those words first, so program order keeps it last.
struct RecSink {
    rsrc_t rs;           // window of the output at byte 4 * wbase
    uint32_t wbase;      // first word of the window
    uint32_t lane;
    uint32_t *stage;  // the wave's 64 scratch words
    uint32_t vrec;    // lane k: record k of the current group
    uint32_t n;       // records in the group (outside the hot loop)
    uint32_t pend;    // bits of the first unfinished output word, MSB-aligned
    uint32_t nb;      // how many (< 32)
    uint32_t wout;    // its word index

    static __device__ __forceinline__ uint32_t scan_add(uint32_t x) { return wave_scan_add(x); }

    // append record rec as number n of the group (outside the hot loop)
    __device__ __forceinline__ void push(uint32_t rec)
    {
        vrec = lane == n ? rec : vrec;
        if (++n == 64) pack();
    }
    // the low n (<= 64) bits of x, MSB first, as records of <= 24 bits
    __device__ void push_bits(uint64_t x, uint32_t nbits)
    {
        while (nbits > 24) {
            nbits -= 24;
            push((1u << 24) | ((uint32_t)(x >> nbits) & 0xFFFFFFu));
        }
        if (nbits) push((1u << nbits) | ((uint32_t)x & ((1u << nbits) - 1u)));
    }

    __device__ void pack()
    {
        const uint32_t rec = lane < n ? vrec : 0u;
        const uint32_t len = rec ? 31u - (uint32_t)__builtin_clz(rec) : 0u;
        const uint32_t code = rec & ((1u << len) - 1u);
        const uint32_t msb = code << ((32u - len) & 31u);  // len 0: code 0
        const uint32_t incl = scan_add(len);
        const uint32_t p = nb + incl - len;  // bit offset in the group's words
        const uint32_t w = p >> 5, o = p & 31u;
        uint32_t head = msb >> o;
        const uint32_t tail = o + len > 32u ? msb << (32u - o) : 0u;
        head |= lane == 0 ? pend : 0u;
        stage[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
        __hip_atomic_fetch_or(&stage[w], head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_or(&stage[w + 1], tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __builtin_amdgcn_wave_barrier();
        const uint32_t word = stage[lane];
        const uint32_t total = nb + lane_read(incl, 63);
        const uint32_t full = total >> 5;  // <= 62
        buf_store(rs, lane < full ? (wout - wbase + lane) * 4 : kDrop, __builtin_bswap32(word));
        pend = lane_read(word, full);
        nb = total & 31u;
        wout += full;
        n = 0;
        __builtin_amdgcn_wave_barrier();
    }

    // the window starts at the current word (stores past cap fall outside every range); called
    // between input chunks (a chunk adds < 2 KB of output)
    __device__ void rebase(uint8_t *out, uint64_t cap)
    {
        wbase = wout;
        const uint64_t at = 4ull * wbase;
        rs = make_rsrc(out + at, at < cap ? (uint32_t)min(cap - at, (uint64_t)kMaxBufBytes) : 0u);
    }

    // pack what is left, zero-pad to a byte (transform.cpp:379-381), store the last 0..4 bytes;
    // returns the byte length
    __device__ __forceinline__ uint64_t finish()
    {
        if (n) pack();
        const uint32_t tail = (nb + 7u) >> 3;  // 0..4 bytes
        for (uint32_t b = 0; b < 4; ++b)
            buf_store8(rs, lane == 0 && b < tail ? (wout - wbase) * 4 + b : kDrop, pend >> (24 - 8 * b));
        return (uint64_t)wout * 4 + tail;
    }
};

// --------------------------------------------------------------------------- the encoder --

// Waves per SIMD each tree layout's LDS admits (8 four-wave workgroups per CU narrow, 6 wide, 4
// huge): the register budget the compiler may use (fewer scalar spills in the wide kernels,
// which C4's single long stream runs)
#ifndef HC_WPE0
#define HC_WPE0 8
#endif
template <int kW, bool kTab = false>
constexpr int kWavesPerSimd = kTab ? (kW == 0 ? 6 : 5) : (kW == 0 ? HC_WPE0 : (kW == 1 ? 6 : 4));

// Which way the encoder finds codes, voted per stream (status[] carries the vote until the
// encoder overwrites it with the stream's status; the two modes' launches run side by side on two
// HIP streams, launch_encode_src): the path cache when the stream's 16 most frequent
// symbols cover most of it (>= 60 %: the diff model's photos, 95 %), the level tables when the
// alphabet is flat (< 9 %: noise, ramps, 6-8 %) -- measured: photo -c -m 8192 streams cache 67
// ms / tables 131, noise -c -m 2048 485 / 227, ramps -c 8192 623 / 365 -- and in between (photos
// without the diff model, 10-13 %; hd01 -c -m 41 %) the tables only when every stream is
// resident at once in table mode's occupancy (photo -c 4096 streams 325 / 231 ms, 8192 401 /
// 436; the 4096^2 -c -a matrix, one stream, 6.25 / 2.97 s; hd01 -c -m alone 108 / 55 ms).
// Estimated from a sample of 16 KB (below): the byte of every run start (diff model applied), a
// 256-bin histogram per wave in LDS, the top 16 by repeated max.
constexpr int32_t kModeTables = -0x7A0, kModeCache = -0x7A1, kModeSmall = -0x7A2;
// small alphabet: at most this many distinct run-start bytes in the sample (grad -c -m: 2)
constexpr uint32_t kSmallVote = 4;
// the small-alphabet steps (encoder code_all_batch, decoder Dec::decode_small): kSmallK symbols
// of kSmallG lanes (levels, depth <= kSmallG) each, while every position is >= kSmallNyt (at
// most 16 symbols seen)
constexpr uint32_t kSmallG = 4, kSmallK = 15, kSmallNyt = kRoot - 32;
template <int kSrc>
__global__ __launch_bounds__(256) void enc_mode_kernel(Batch bt, uint32_t low_occ, uint32_t forced)
{
    __shared__ uint32_t hist[4][256];
    const uint32_t lane = lane_id(), wv = uni(threadIdx.x >> 6);
    const uint32_t sid = blockIdx.x * 4 + wv;
    if (sid >= bt.n) return;
    if (forced) {
        if (lane == 0) bt.status[sid] = forced == 2 ? kModeTables : (forced == 3 ? kModeSmall : kModeCache);
        return;
    }
    uint32_t *h = hist[wv];
    for (uint32_t i = lane; i < 256; i += 64) h[i] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint64_t n = bt.in_lens[sid];
    const uint8_t *const in = bt.in + bt.in_offs[sid];
    // The sample: a stream of <= 16 KB whole, a longer one as 64 segments of 256 bytes spread
    // evenly over it (its first 16 KB alone misjudged hd01 -c -m, a flat top and then a wide
    // alphabet: cache 108 ms against tables 55 ms as a lone stream). Four bytes per lane and
    // segment, one dword load (the bytes of a last dword past the stream masked off); each byte's
    // previous byte comes from the dword before (lane - 1, lane 63 of the segment before when they
    // are contiguous, else the byte before the segment) and a spread segment's first symbol
    // starts a run.
    const bool spread = n > 16384;
    const uint32_t nseg = spread ? 64u : (uint32_t)((n + 255) / 256);
    uint32_t prev_raw = 0, prev_sym = 0, total = 0;  // lane 63's dwords of the last segment; run starts
#if HC_VOTE_BATCH
    // the spread segments are independent (each one's first symbol starts a run, its previous raw
    // byte is the byte before it): kVB segments' loads go out together, then their histogram
    // updates (one at a time, each waiting for its load, the vote was 64 global round trips long:
    // 0.11 ms of grad's 1.25 ms encode)
    if (spread) {
        constexpr uint32_t kVB = 8;
        // segment k starts at ((n - 256) k / 63) & ~3, stepped without a 64-bit division per
        // segment (the scalar unit has none: each was a long SALU sequence, 70 SALU a segment)
        const uint64_t q = uni64((n - 256) / 63);
        const uint32_t r = uni((uint32_t)((n - 256) - 63 * q));
        uint64_t ob = 0;   // q k + (r k) / 63
        uint32_t oa = 0;   // (r k) % 63
        for (uint32_t k0 = 0; k0 < 64; k0 += kVB) {
            uint32_t w[kVB], pr[kVB];
#pragma unroll
            for (uint32_t u = 0; u < kVB; ++u) {
                const uint64_t o = ob & ~3ull;
                ob += q;
                oa += r;
                if (oa >= 63) {
                    oa -= 63;
                    ++ob;
                }
                w[u] = buf_load(make_rsrc(in + o, 256u), 4 * lane);
                // the dword ending at the segment's first byte (its top byte: the byte before)
                // (no branch: a load under one would be waited for at the join)
                pr[u] = buf_load(make_rsrc(in + (o ? o - 4 : 0), 4u), 0u) & (o ? 0xFF000000u : 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < kVB; ++u) {
                uint32_t sy = w[u];
                if (kSrc == SRC_RAW_DIFF) {  // transform.cpp:220-229 (m[-1] = 0), bytewise
                    const uint32_t xp = (w[u] << 8) | (wave_shr1(w[u], pr[u]) >> 24);
                    sy = ((w[u] | 0x80808080u) - (xp & 0x7F7F7F7Fu)) ^ ((w[u] ^ ~xp) & 0x80808080u);
                }
                const uint32_t sp = (sy << 8) | (wave_shr1(sy, 0u) >> 24);
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t i = 4 * lane + j, v = byte_of(sy, j);
                    const bool start = i == 0 || v != byte_of(sp, j);
                    if (start) atomicAdd(&h[v], 1u);
                    total += (uint32_t)__builtin_popcountll(ballot(start));
                }
            }
        }
    }
    for (uint32_t k = 0; k < (spread ? 0u : nseg); ++k) {
#else
    for (uint32_t k = 0; k < nseg; ++k) {
#endif
        const uint64_t o = spread ? ((n - 256) * k / 63) & ~3ull : 256ull * k;
        const uint32_t len = (uint32_t)min(n - o, (uint64_t)256);
        const uint32_t w = buf_load(make_rsrc(in + o, (len + 3u) & ~3u), 4 * lane);
        if (spread) prev_raw = o ? (uint32_t)in[o - 1] << 24 : 0u;
        uint32_t sy = w;
        if (kSrc == SRC_RAW_DIFF) {  // transform.cpp:220-229 (m[-1] = 0), bytewise
            const uint32_t xp = (w << 8) | (wave_shr1(w, prev_raw) >> 24);
            sy = ((w | 0x80808080u) - (xp & 0x7F7F7F7Fu)) ^ ((w ^ ~xp) & 0x80808080u);
            prev_raw = lane_read(w, 63);
        }
        const uint32_t sp = (sy << 8) | (wave_shr1(sy, prev_sym) >> 24);
        prev_sym = lane_read(sy, 63);
        const bool first = spread || k == 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t i = 4 * lane + j, v = byte_of(sy, j);
            const bool start = i < len && ((first && i == 0) || v != byte_of(sp, j));
            if (start) atomicAdd(&h[v], 1u);
            total += (uint32_t)__builtin_popcountll(ballot(start));
        }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t c[4], top = 0;
    for (uint32_t k = 0; k < 4; ++k) c[k] = h[64 * k + lane];
    for (uint32_t r = 0; r < 16; ++r) {
        uint32_t mx = max(max(c[0], c[1]), max(c[2], c[3]));
        for (uint32_t d = 32; d; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
        top += mx;
        const uint64_t who = ballot(c[0] == mx || c[1] == mx || c[2] == mx || c[3] == mx);
        if (lane == (uint32_t)__builtin_ctzll(who)) {  // take out one of the maxima
            if (c[0] == mx) c[0] = 0;
            else if (c[1] == mx) c[1] = 0;
            else if (c[2] == mx) c[2] = 0;
            else c[3] = 0;
        }
    }
    const bool cache = total == 0 || 100ull * top >= 60ull * total || (100ull * top >= 9ull * total && !low_occ);
    // the distinct run-start bytes: at most kSmallVote -> the small-alphabet launch (whose steps
    // need <= 16 FGK symbols; a stream whose count bytes widen the alphabet falls back to the
    // regular batches there)
    uint32_t distinct = 0;
    for (uint32_t k = 0; k < 4; ++k) distinct += (uint32_t)__builtin_popcountll(ballot(h[64 * k + lane] != 0));
    const bool small = total != 0 && distinct <= kSmallVote;
    if (lane == 0) bt.status[sid] = small ? kModeSmall : (cache ? kModeCache : kModeTables);
}

template <int kW, int kSrc, bool kTab = false, bool kSmall = false>
__global__ __launch_bounds__(64 * HC_WAVES) __attribute__((amdgpu_waves_per_eu(kWavesPerSimd<kW, kTab>))) void encode_kernel(Batch bt)
{
    __shared__ Tree<kW, false, kTab, kSmall> trees[kWaves];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t sid = blockIdx.x * kWaves + wv;
    if (sid >= bt.n) return;
    uint64_t pacc = 0;  // HC_PROF regions
    (void)pacc;

    const uint64_t in_off = uni64(bt.in_offs[sid]);
    const uint64_t n = uni64(bt.in_lens[sid]);
    const uint64_t out_off = uni64(bt.out_offs[sid]);
    const uint64_t cap = uni64(bt.out_caps[sid]);

    // the worst-case symbol count (MNP-5 expands by at most 4/3) decides the tree layout; the
    // other layouts' launches skip the stream
    const uint64_t max_sym = kSrc == SRC_SYMBOLS ? n : n + n / 3 + 2;
    if (tree_kind(max_sym, bt.min_tree) != (uint32_t)kW) return;
    // narrow and wide: the cache, table and (narrow) small-alphabet launches split the streams
    // (enc_mode_kernel; a wide stream voted small takes the cache launch)
    if (kW <= 1) {
        const int32_t mode = (int32_t)uni((uint32_t)bt.status[sid]);
        if ((mode == kModeTables) != kTab || (kW == 0 && mode == kModeSmall) != kSmall) return;
    }
    const uint32_t window = window_bytes();

    Fgk<kW, false, kTab, kSmall> fgk(trees[wv], lane);
    RecSink sink;
    sink.rs = make_rsrc(bt.out + out_off, (uint32_t)min(cap, (uint64_t)kMaxBufBytes));
    sink.wbase = 0;
    sink.lane = lane;
    sink.stage = fgk.T.scratch;
    sink.vrec = 0;
    sink.n = 0;
    // headers.cpp:118-122: the flags byte opens word 2 (words 0-1: the u64 symbol count,
    // written at the end)
    const uint32_t flags = kSrc == SRC_SYMBOLS ? bt.flags : (kSrc == SRC_RAW_DIFF ? 0x80u : 0u);
    sink.pend = flags << 24;
    sink.nb = 8;
    sink.wout = 2;

    // input: 256-byte chunks ci < nch through a window; ioff = the next load's offset in it
    rsrc_t rin = make_rsrc(bt.in + in_off, (uint32_t)min((n + 3u) & ~3ull, (uint64_t)kMaxBufBytes));
    const uint32_t nch = (uint32_t)((n + 255) / 256);
    uint32_t ioff = 256;

    // transform.cpp:363-384: per symbol encode (path before update), then update. A symbol
    // whose root path is cached (the common case) takes the hot path, written so that its
    // wave-uniform values stay in VGPRs (the scalar unit is shared by the CU's 32 waves): the
    // symbol's path-cache row, the lane-parallel update, its record in lane t - koff. Anything
    // else (a symbol not cached, or unseen) takes the miss path, which appends its records
    // through the sink and re-bases koff. Positions stay in range by construction, so `bad` (a
    // bug detector) is checked once per chunk.
    const uint8_t *const sb = reinterpret_cast<const uint8_t *>(fgk.T.syms);
    uint8_t *const sb_w = reinterpret_cast<uint8_t *>(fgk.T.syms);
    auto miss = [&](uint32_t sv) {
        const uint32_t sym = uni(sv);
        uint32_t s = uni(fgk.T.where[sym]) & 1023u;
        const uint32_t fresh = s == 0;
        if (fresh) s = uni(fgk.split(sym));
        uint32_t pv;
        uint32_t d;
        {
            HC_PROF_BEGIN();
            d = fgk.chase(s, pv);
            HC_PROF_END(5);
        }
        // bit k = code bit (position parity, left = even) of level k; read MSB first it is the
        // root-to-leaf code (the kRoot lanes are even)
        const uint64_t bits = ballot(pv & 1u);
        if (d <= kInsertDepth) fgk.pc_insert(sym, s, pv, d, (1u << d) | (uint32_t)bits);
        {
            HC_PROF_BEGIN();
            // a path too deep to cache belongs to a rare symbol, whose leaf nearly always ties
            // with the next position (9 in 10 on the slot-form model): walk from the leaf at once
            if (d > kInsertDepth) {
                fgk.pc_bound();
                fgk.walk(s, pv, true);
            }
            else fgk.update_path(pv);
            HC_PROF_END(6);
        }
        if (fresh) {
            // the path starts at the new leaf, one level below the NYT whose code is sent
            // (huffman.cpp:44-50): drop that lowest bit, then 8 raw bits
            sink.push_bits(bits >> 1, d - 1);
            sink.push((1u << 8) | sym);
        } else {
            sink.push_bits(bits, d);
        }
    };
    // code symbols syms[0..ns) of the LDS buffer. The hot loop carries only vt, the records, the
    // cache's reference bits and its read pipeline: a miss or a failed leader test leaves it
    // (what = 1 / 2) and is finished outside, so the compiler adds no copies of the rare paths'
    // state per symbol. Pipeline: while symbol t updates, the cache row of t+1, the where[]
    // entry of t+2 and the byte of t+3 are already in flight. where[] and the rows change only
    // on the paths that leave the loop (split, insert, swap), so what was read ahead stays
    // valid inside it; the loop is re-primed after every exit. Bytes past ns are older symbols
    // of the same buffer: their reads are harmless.
    auto code_all = [&](uint32_t ns) __attribute__((always_inline)) {
        uint32_t t = 0;
        while (t < ns) {
            uint32_t rl = sink.n;  // record lane of symbol t (scalar)
            const uint32_t rend = min(64u, rl + (ns - t));
            uint32_t vt = vreg(t);
            uint32_t ws0 = vreg(fgk.T.where[sb[vt]]);      // where[] entry of symbol t
            uint32_t ws1 = vreg(fgk.T.where[sb[vt + 1]]);  // ... of t+1
            uint32_t e0 = ws0 >> 10;
            uint32_t pr0 = vreg(fgk.pc_lane[e0 * kRow]);   // cache row of t (pc_miss if none)
            uint32_t sv2 = vreg(sb[vt + 2]);               // byte of t+2
            // LDS address of the byte of t+3, in a VGPR (one add per symbol, no base add)
            const lds_u8 *vb = (const lds_u8 *)sb + t + 3;
            asm("" : "+v"(vb));
            uint32_t pv, k;
            // loop while no level failed (k = 0xFFFFFFFF) and record lanes are left (left < 0):
            // both sign bits set, one scalar AND
            int32_t left = (int32_t)(rl - rend);
            do {
                const uint32_t rec = fgk.pc_use(e0, pr0, pv);
                k = fgk.update_fast(pv, [&] {
                    // (v_bfe + v_lshl_add; left alone the compiler emits shift, and, add)
                    const uint32_t pr1 = fgk.pc_lane[opaque(__builtin_amdgcn_ubfe(ws1, 10, 6)) * kRow];
                    const uint32_t ws2 = fgk.T.where[sv2];
                    const uint32_t sv3 = *vb;
                    pr0 = pr1;
                    ws1 = ws2;
                    sv2 = sv3;
                });
                sink.vrec = writelane(sink.vrec, rec, (uint32_t)((int32_t)rend + left));
                ++vb;
                ++left;
            } while ((int32_t)(k & (uint32_t)left) < 0);
            rl = (uint32_t)((int32_t)rend + left);
            t += rl - sink.n;
            if (k != 0xFFFFFFFFu) {
                // not cached (the miss row's sentinel at level 0): nothing was written; code it
                // from scratch
                if (lane_read(pv, 0) == kMissPos) {
                    --t;
                    sink.n = rl - 1;  // its record lane, overwritten by the miss path
                    HC_PROF_BEGIN();
                    miss(sb[t]);
                    HC_PROF_END(1);
                    ++t;
                    continue;
                }
                HC_PROF_BEGIN();
                fgk.walk(lane_read(pv, k), pv);
                HC_PROF_END(2);
            }
            sink.n = rl;
            if (rl == 64) {
#ifndef HC_PROF_PASS
                HC_PROF_BEGIN();
                sink.pack();
                HC_PROF_END(3);
#else
                sink.pack();
#endif
            }
        }
    };

    // Batched hot path (path-cache mode, narrow and wide layouts, HC_ENC_BATCH; model:
    // tests/fgk_batch_model.py, test tests/test_batch_model.py).
    // Between swaps and splits the tree's shape is fixed and an update only adds 1 to the
    // weights on the symbol's root path, so the updates of consecutive cached symbols commute.
    // Seven symbols at a time, lane 9 j + l taking level l of symbol j's cached path (level d =
    // its depth: the root, counted once; l > d: root padding), the decoder's tentative commit
    // (Dec::decode_batch):
    //  1. every path position of every batch symbol gets its increment (one LDS add: +1024 to the
    //     narrow weight word, +1 to a wide weight, the root once per symbol), the words of the
    //     next positions having been read before;
    //  2. a level fails when that next word is below the position's word after the adds -- the
    //     one-symbol loop's update_fast test with every batch symbol through the position counted
    //     as earlier and none through the next one, so it reports levels falsely at worst (the
    //     exact counts, from membership bits ORed into the body words, measured 394 ms on C5
    //     where this takes 371);
    //  3. the first symbol with a failed level or without a cached path (the miss row's kMissPos)
    //     ends the batch: its increments and those after it are taken back, the code records of
    //     the ones before it go to the sink, and it is coded alone (miss / update_path: walk).
    //     Without such a symbol (the empty failure mask's ff1 is 0xFFFFFFFF) jf clamps to jmax;
    //     idle lane 63 holds the root, which never fails.
    // Per symbol ~10 instructions where the one-symbol loop takes ~26, and one dependent chain of
    // LDS round trips per batch instead of per symbol.
    // seven symbols in groups of nine lanes (levels 0..8: every cached path), the root's
    // increments by lane 63 in the same adds (measured: six symbols in groups of ten, the root in
    // each group, C5 encode 369 ms against 349)
    // Small alphabets (narrow layout, while at most 16 symbols are seen, so every position is >=
    // 480; model: tests/fgk_batch_model.py small_len, encode(small=True)). A run-heavy stream with a
    // few symbols (grad -c -m: 1, 3, 250, 255) ties on every row, and the tentative test below
    // counts no earlier batch symbol through the next position: it ends a batch every ~4 symbols
    // (1034 batches and 523 symbols alone per 512x512 stream). Here the counts are exact and the
    // paths short, so up to 15 symbols go per step, four lanes each (levels 0..3: depth <= 4;
    // lane 63 holds the root): every path position ORs its symbol's bit into a membership mark
    // (smark, 2 positions per word), and symbol j's test at position a reads the pre-batch words
    // of a and a + 1 and the marks of both: with c0 / c1 the earlier symbols through a / a + 1
    // (c1 = j at the root: every symbol passes it) the level passes iff weight(a + 1) + c1 >=
    // weight(a) + c0 + 1 -- the one-symbol loop's leader test on the tree as the earlier symbols
    // leave it. The first symbol with a failing level (or no cached path, or a path deeper than
    // four) ends the step: the ones before it commit with one add, it is coded alone. grad:
    // 319 steps and 13 symbols alone per stream. Returns where the regular batches take over.
    constexpr uint32_t kSG = kSmallG, kSK = kSmallK;
    constexpr uint32_t kBatch = 7, kLv = 9;  // (the masks: groups9)
    static_assert(kBatch * kLv <= 63 && kLv >= kInsertDepth, "batch lanes: every cached path, lane 63 free");
    constexpr uint32_t kIncU = kW ? 1u : 1024u;
    auto code_all_batch = [&](uint32_t ns) __attribute__((always_inline)) {
        const uint32_t bj = lane < kBatch * kLv ? lane / kLv : 7u;  // the lane's symbol (7: idle)
        const uint32_t bl = lane < kBatch * kLv ? lane % kLv : 0u;  // ... and level
        const uint64_t idle = ~0ull << (kBatch * kLv);
        const uint32_t rowb = lds_off16(&fgk.T.pc[0]) + 2 * bl - 2 * kRow;  // + 32 e: row e - 1 (e = 0: pc_miss)
        const uint32_t wtb = lds_off(&fgk.T.wt[0]);
        const uint32_t whb = lds_off16(&fgk.T.where[0]);
        const uint32_t scb = lds_off(fgk.scr32());
        const uint32_t svb = (uint32_t)(size_t)(const lds_u8 *)sb + bj;
        const uint32_t lkl = lane * kLv;
        constexpr uint64_t kL63 = 1ull << 63;
        uint32_t t = 0;
        // small-alphabet steps (above) while the stream has seen <= 16 symbols; re-checked only
        // after a symbol coded alone (splits happen there), so a regular step pays nothing for it
        if constexpr (!kSmall) {
            // (the path-cache kernel: one regular batch step per pass of this loop)
            while (t < ns) {
                uint32_t jf, jmax;
                if (sink.n > 64 - kBatch) sink.pack();
                HC_CNT(1);
                jmax = min(kBatch, ns - t);
                const uint32_t sv = opaque(*(const lds_u8 *)(size_t)(svb + t));
                const uint32_t wh = opaque(*(const lds_u16 *)(size_t)(whb + 2 * sv));
                const uint32_t e = wh >> 10;
                uint32_t pos = opaque(*(const lds_u16 *)(size_t)(rowb + 32 * e));
                // lane 63 (idle) holds the root and adds one increment per batch symbol
                pos = sel(idle, kRoot, pos);
                const uint32_t wa = wtb + 4 * pos;
                const uint64_t am = (ballot(pos < kRoot) & groups9(jmax)) | (jmax ? kL63 : 0);
                const uint32_t vinc = sel(kL63, jmax * kIncU, kIncU);
                // 1. tentative increments (each path position once, the root once per symbol)
                const uint32_t w1 = *(const lds_u32 *)(size_t)(wa + 4);
                __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(am, wa, scb), vinc, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WAVEFRONT);
                const uint32_t wn = *(const lds_u32 *)(size_t)wa;
                // 2. the tests; 3. the increments from the first failing symbol on taken back
                const uint64_t fm = (ballot(w1 < wn) & am) | ballot(pos == kMissPos);
                jf = min(ff1(fm) / kLv, jmax);  // the failing lane's symbol
                if (jf < jmax) {
                    const uint32_t vdec = sel(kL63, (jf - jmax) * kIncU, 0u - kIncU);
                    __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(am & ~groups9(jf), wa, scb),
                                           vdec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
                const uint32_t q = lane - sink.n;  // record lane q of the batch: symbol q's record
                // the code record 1 << d | bits (bit k: level k's parity, left = even) from two
                // ballots: the group's parity bits below its first root lane
                const uint64_t par = ballot(pos & 1u), rtm = ballot(pos == kRoot);
                const uint32_t gb = lkl - sink.n * kLv;  // q * kLv
                const uint32_t d = (uint32_t)__builtin_ctz((uint32_t)(rtm >> gb) | (1u << kLv));
                const uint32_t r = __builtin_amdgcn_ubfe((uint32_t)(par >> gb), 0, d) | (1u << d);
                sink.vrec = q < jf ? r : sink.vrec;
                __builtin_amdgcn_wave_barrier();
                sink.n += jf;
                t += jf;
                if (jf < jmax) {  // symbol t: not cached, or a level reported (small: deeper than 4): alone
                    HC_CNT(2);
                    if (sink.n == 64) sink.pack();
                    const uint32_t sym = uni(sb[t]);
                    const uint32_t ent = uni(fgk.T.where[sym]) >> 10;
                    if (ent == 0) {
                        HC_PROF_BEGIN();
                        miss(sym);
                        HC_PROF_END(1);
                    } else {
                        HC_PROF_BEGIN();
                        uint32_t pv;
                        const uint32_t rc = fgk.pc_use(ent, fgk.pc_lane[ent * kRow], pv);
                        sink.push(rc);
                        fgk.update_path(pv);
                        HC_PROF_END(2);
                    }
                    ++t;
                }
            }
        } else {
            bool small = fgk.nyt >= kSmallNyt;
            while (t < ns) {
                uint32_t jf, jmax;
                if (small) {
                    // (the lane index opaque: these per-lane values are made here, not hoisted to the
                    // kernel's entry beside the regular step's)
                    const uint32_t ln = vreg(lane);
                    const uint32_t g = ln < kSK * kSG ? ln >> 2 : kSK;  // the lane's symbol (kSK: idle)
                    const uint32_t srow = lds_off16(&fgk.T.pc[0]) + 2 * (ln & 3u) - 2 * kRow;
                    const uint32_t ssv = (uint32_t)(size_t)(const lds_u8 *)sb + (g < kSK ? g : 0u);
                    const uint32_t sscb = lds_off(&fgk.T.scratch[0]) + 4 * ln;
                    const uint32_t mkb = lds_off(&fgk.T.smark[0]);
                    // the cached path of the step's symbols: symbol byte -> where[] -> row (level
                    // 4 too, for the depth test). (Measured: read one step ahead, for the step
                    // that follows if this one takes all its symbols -- rows and where[] change
                    // only on the alone path -- grad encode 1.28 -> 1.33 ms.)
                    auto row_read = [&](uint32_t t0, uint32_t &p4v) __attribute__((always_inline)) {
                        const uint32_t sv = opaque(*(const lds_u8 *)(size_t)(ssv + t0));
                        const uint32_t wh = opaque(*(const lds_u16 *)(size_t)(whb + 2 * sv));
                        const uint32_t ra = srow + 32 * (wh >> 10);
                        p4v = opaque(*(const lds_u16 *)(size_t)(ra + 8));  // lane l = 0: level 4
                        return opaque(*(const lds_u16 *)(size_t)ra);
                    };
                    do {
                        if (sink.n > 64 - kSK) sink.pack();
                        HC_CNT(1);
                        jmax = min(kSK, ns - t);
                        uint32_t p4, pos = row_read(t, p4);
                        pos = sel(~0ull << (kSK * kSG), kRoot, pos);
                        const uint32_t wa = wtb + 4 * pos;
                        const uint64_t gm = below_mask(kSG * jmax);
                        const uint64_t am = ballot(pos < kRoot) & gm;
                        // no cached path, or one deeper than four: the step ends there
                        const uint64_t em = (ballot(pos == kMissPos) | ballot((ln & 3u) == 0 && p4 != kRoot)) & gm;
                        const uint32_t w0 = *(const lds_u32 *)(size_t)wa, w1 = *(const lds_u32 *)(size_t)(wa + 4);
                        const uint32_t ma = pos - kSmallNyt, odd = ma & 1u;  // (pos >= 480 on the am lanes)
                        const uint32_t mda = sel(am, mkb + 4 * (ma >> 1), sscb);
                        __hip_atomic_fetch_or((uint32_t *)(lds_u32 *)(size_t)mda, (1u << g) << (odd << 4),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        // the marks of a (half `odd` of its word) and a + 1 (the other half, or the next word)
                        const uint32_t mlo = *(const lds_u32 *)(size_t)mda;
                        const uint32_t mhi = *(const lds_u32 *)(size_t)(mda + 4 * odd);
                        const uint32_t c0 = (uint32_t)__builtin_popcount(__builtin_amdgcn_ubfe(mlo, odd << 4, g));
                        const uint32_t c1 = pos + 1 == kRoot ? g
                                                             : (uint32_t)__builtin_popcount(__builtin_amdgcn_ubfe(odd ? mhi : mlo, (odd ^ 1u) << 4, g));
                        const uint64_t fm = (ballot((w1 >> 10) + c1 < (w0 >> 10) + c0 + 1) & am) | em;
                        jf = min(ff1(fm) >> 2, jmax);
                        // symbols < jf commit (+1 per path position and symbol, the root once each: lane
                        // 63); the marks are cleared
                        __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel((am & below_mask(kSG * jf)) | kL63, wa, sscb),
                                               sel(kL63, jf << 10, 1u << 10), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        *(lds_u32 *)(size_t)mda = 0u;
                        // code records (as below): record lane sink.n + q takes symbol q's
                        const uint32_t q = ln - sink.n;
                        const uint64_t par = ballot(pos & 1u), rtm = ballot(pos == kRoot);
                        const uint32_t gb = kSG * q;
                        const uint32_t d = (uint32_t)__builtin_ctz((uint32_t)(rtm >> gb) | (1u << kSG));
                        const uint32_t r = __builtin_amdgcn_ubfe((uint32_t)(par >> gb), 0, d) | (1u << d);
                        sink.vrec = q < jf ? r : sink.vrec;
                        __builtin_amdgcn_wave_barrier();
                        sink.n += jf;
                        t += jf;
                    } while (jf == jmax && t < ns);
                } else {
                    do {
                        if (sink.n > 64 - kBatch) sink.pack();
                        HC_CNT(1);
                        jmax = min(kBatch, ns - t);
                        const uint32_t sv = opaque(*(const lds_u8 *)(size_t)(svb + t));
                        const uint32_t wh = opaque(*(const lds_u16 *)(size_t)(whb + 2 * sv));
                        const uint32_t e = wh >> 10;
                        uint32_t pos = opaque(*(const lds_u16 *)(size_t)(rowb + 32 * e));
                        // lane 63 (idle) holds the root and adds one increment per batch symbol
                        pos = sel(idle, kRoot, pos);
                        const uint32_t wa = wtb + 4 * pos;
                        const uint64_t am = (ballot(pos < kRoot) & groups9(jmax)) | (jmax ? kL63 : 0);
                        const uint32_t vinc = sel(kL63, jmax * kIncU, kIncU);
                        // 1. tentative increments (each path position once, the root once per symbol)
                        const uint32_t w1 = *(const lds_u32 *)(size_t)(wa + 4);
                        __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(am, wa, scb), vinc, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WAVEFRONT);
                        const uint32_t wn = *(const lds_u32 *)(size_t)wa;
                        // 2. the tests; 3. the increments from the first failing symbol on taken back
                        const uint64_t fm = (ballot(w1 < wn) & am) | ballot(pos == kMissPos);
                        jf = min(ff1(fm) / kLv, jmax);  // the failing lane's symbol
                        if (jf < jmax) {
                            const uint32_t vdec = sel(kL63, (jf - jmax) * kIncU, 0u - kIncU);
                            __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(am & ~groups9(jf), wa, scb),
                                                   vdec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                        const uint32_t q = lane - sink.n;  // record lane q of the batch: symbol q's record
                        // the code record 1 << d | bits (bit k: level k's parity, left = even) from two
                        // ballots: the group's parity bits below its first root lane
                        const uint64_t par = ballot(pos & 1u), rtm = ballot(pos == kRoot);
                        const uint32_t gb = lkl - sink.n * kLv;  // q * kLv
                        const uint32_t d = (uint32_t)__builtin_ctz((uint32_t)(rtm >> gb) | (1u << kLv));
                        const uint32_t r = __builtin_amdgcn_ubfe((uint32_t)(par >> gb), 0, d) | (1u << d);
                        sink.vrec = q < jf ? r : sink.vrec;
                        __builtin_amdgcn_wave_barrier();
                        sink.n += jf;
                        t += jf;
                    } while (jf == jmax && t < ns);
                }
                if (jf < jmax) {  // symbol t: not cached, or a level reported (small: deeper than 4): alone
                    HC_CNT(2);
                    if (sink.n == 64) sink.pack();
                    const uint32_t sym = uni(sb[t]);
                    const uint32_t ent = uni(fgk.T.where[sym]) >> 10;
                    if (ent == 0) {
                        HC_PROF_BEGIN();
                        miss(sym);
                        HC_PROF_END(1);
                    } else {
                        HC_PROF_BEGIN();
                        uint32_t pv;
                        const uint32_t rc = fgk.pc_use(ent, fgk.pc_lane[ent * kRow], pv);
                        sink.push(rc);
                        fgk.update_path(pv);
                        HC_PROF_END(2);
                    }
                    ++t;
                    small = kSmall && fgk.nyt >= kSmallNyt;
                }
            }
        }
    };

    // Table mode (kTab): no path cache. The decoder's level tables (levels 1..8, prefix ->
    // where the walk from the root stops) and pcode[] (position -> the code the tables reached
    // it by) give a symbol's code and whole root path from three reads: where[] -> pcode[] ->
    // one lane-parallel read of the tables (lane k: level 8 - k), exactly the decoder's path
    // read. The level-8 entry read back must name the symbol's own position at the pcode depth;
    // otherwise (deeper than 8, or not in the tables since a split) the symbol is coded from
    // scratch like a cache miss. A symbol's reads go out up to three symbols ahead (where[],
    // pcode[] and the tables change only on the paths that leave the loop).
    const uint32_t psh = lane < 8 ? lane : 8u;
    const uint32_t pbase = lds_off16(&fgk.T.lvl[0]) + 2 * (lane < 8 ? (256u >> lane) - 2 : 0xFFFFFFFEu);
    auto path_read = [&](uint32_t pcw) __attribute__((always_inline)) {
        return opaque(*(const lds_u16 *)(size_t)(pbase + ((pcw & 255u) >> psh) * 2));
    };
    // the root path of position s0 (lane k: level k, kRoot above): climb parent links until a
    // position that pcode[] puts at depth 8 and the tables confirm; the tables give the other 8
    // levels in one read (a 10-bit code: 2 climbs instead of 10). Returns the depth.
    auto chase_tab = [&](uint32_t s0, uint32_t &pv) __attribute__((always_inline)) -> uint32_t {
        uint32_t s = s0, n = 0, td = kRoot;  // td lane j: level n - 1 - j
        for (;;) {
            const uint32_t pc = uni(fgk.T.pcode[s]);
            const uint32_t par = fgk.parent(s);
            if (((pc >> 8) & 7u) == 7u) {
                const uint32_t pr = path_read(pc);
                if (uni(pr) == (s | (8u << 10))) {
                    const uint32_t dn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((n - 1 - lane) & 63u) * 4), (int)td);
                    const uint32_t tb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - n) & 63u) * 4), (int)pr);
                    pv = lane < n ? dn : (lane - n < 9 ? (tb & 1023u) : kRoot);
                    return n + 8;
                }
            }
            const uint32_t sh = __builtin_amdgcn_update_dpp(0u, td, 0x138, 0xF, 0xF, true);
            td = lane == 0 ? s : sh;
            ++n;
            if (par == kRoot || n >= 63) {  // the root, or (a bug) a cycle
                fgk.bad |= par ^ kRoot;
                const uint32_t dn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((n - 1 - lane) & 63u) * 4), (int)td);
                pv = lane < n ? dn : kRoot;
                return n;
            }
            s = par;
        }
    };
    auto miss_tab = [&](uint32_t sv) {
        const uint32_t sym = uni(sv);
        uint32_t s = uni(fgk.T.where[sym]) & 1023u;
        const uint32_t fresh = s == 0;
        if (fresh) s = uni(fgk.split(sym));
        uint32_t pv;
        uint32_t d;
        {
            HC_PROF_BEGIN();
            d = chase_tab(s, pv);
            HC_PROF_END(6);
        }
        const uint64_t bits = ballot(pv & 1u);
        if (!fresh && d <= 8) {  // the tables are short of it (a split since the last build)
            if (++fgk.stale >= kRefresh) fgk.from = 0;
        }
        HC_PROF_BEGIN();
        if (d > kInsertDepth) fgk.walk(s, pv);
        else fgk.update_path(pv);
        HC_PROF_END(7);
        if (fresh) {
            sink.push_bits(bits >> 1, d - 1);
            sink.push((1u << 8) | sym);
        } else {
            sink.push_bits(bits, d);
        }
    };
    auto code_all_tab = [&](uint32_t ns) __attribute__((always_inline)) {
        uint32_t t = 0;
        while (t < ns) {
            if (fgk.from < 9) {
                HC_PROF_BEGIN();
                fgk.build_levels();
                HC_PROF_END(5);
            }
            uint32_t rl = sink.n;
            const uint32_t rend = min(64u, rl + (ns - t));
            const uint32_t x1 = vreg(fgk.T.where[sb[t + 1]]);
            const uint32_t x0 = vreg(fgk.T.where[sb[t]]);
            uint32_t pc0 = vreg(fgk.T.pcode[x0 & 1023u]);   // pcode of t
            uint32_t pr = path_read(pc0);                      // path of t
            uint32_t x0u = x0;
            uint32_t pc1 = vreg(fgk.T.pcode[x1 & 1023u]);   // pcode of t+1
            uint32_t x1u = x1;
            uint32_t x2 = vreg(fgk.T.where[sb[t + 2]]);      // where[] of t+2
            uint32_t sv3 = vreg(sb[t + 3]);                    // byte of t+3
            const lds_u8 *vb = (const lds_u8 *)sb + t + 4;
            asm("" : "+v"(vb));
            uint32_t pv, k, ok;
            int32_t left = (int32_t)(rl - rend);
            do {
                const uint32_t pcu = uni(pc0);
                const uint32_t d = ((pcu >> 8) & 7u) + 1;
                ok = uni(pr) == ((uni(x0u) & 1023u) | (d << 10));
                const uint32_t rec = (1u << d) | ((pcu & 255u) >> (8 - d));
                pv = pr & 1023u;
                uint32_t prn;
                k = fgk.update_fast(pv, [&] {
                    prn = path_read(pc1);
                    const uint32_t pc2 = fgk.T.pcode[x2 & 1023u];
                    const uint32_t x3 = fgk.T.where[sv3];
                    const uint32_t sv4 = *vb;
                    x0u = x1u;
                    x1u = x2;
                    pc0 = pc1;
                    pc1 = pc2;
                    x2 = x3;
                    sv3 = sv4;
                }, ok ? 0u : 0xFFFFFFFFu);
                pr = prn;
                sink.vrec = writelane(sink.vrec, rec, (uint32_t)((int32_t)rend + left));
                ++vb;
                ++left;
            } while ((int32_t)(k & (uint32_t)left) < 0);
            rl = (uint32_t)((int32_t)rend + left);
            t += rl - sink.n;
            if (k != 0xFFFFFFFFu) {
                if (!ok) {  // not in the tables: nothing was stored; code it from scratch
                    --t;
                    sink.n = rl - 1;  // its record lane, overwritten by the miss path
                    HC_PROF_BEGIN();
                    miss_tab(sb[t]);
                    HC_PROF_END(1);
                    ++t;
                    continue;
                }
                HC_PROF_BEGIN();
                fgk.walk(lane_read(pv, k), pv);
                HC_PROF_END(2);
            }
            sink.n = rl;
            if (rl == 64) {
#ifndef HC_PROF_PASS
                HC_PROF_BEGIN();
                sink.pack();
                HC_PROF_END(3);
#else
                sink.pack();
#endif
            }
        }
    };

    uint64_t nsym = 0;
    uint32_t next = buf_load(rin, lane * 4);
    RleCarry cy = {0, 0, 0};
    // Two copies of the chunk loop: streams that fit one window (every batch stream) run without
    // the window bookkeeping, which would otherwise sit in scalar registers across the hot loop,
    // and let the MNP-5 symbols of many chunks gather in syms[] before the FGK loop codes them (a
    // run-heavy stream yields a few symbols per chunk: one coding pass per buffer instead of per
    // chunk; grad -c -m encode 3.77 -> 2.89 ms, photo unchanged).
    auto chunks = [&](auto windowed) __attribute__((always_inline)) {
        constexpr bool kWin = decltype(windowed)::value;
        Prio<uint32_t> prio;
        uint32_t np = 0;       // symbols pending in syms[]
        uint32_t chunk = 0;
        bool redo = false;     // the chunk did not fit the pending symbols: again, after coding them
        // Run-heavy stretches (a 256-byte chunk whose run starts sit in at most kSparseEnter
        // lanes) switch to blocks of kQ KB coded by segments (rle_block; tests/rle_chunk_model.py:
        // rle_blocked) while the blocks stay sparse and a whole block of full chunks remains before
        // the last one; blk holds the block at ci (kQ 16-byte loads per lane, the next block in
        // flight).
        constexpr bool kSparseOn = HC_SPARSE && !kWin && kSrc != SRC_SYMBOLS && !kTab;
        constexpr uint32_t kSparseEnter = 2;
        constexpr uint32_t kQ = HC_SPARSE_KB, kBC = 4 * kQ;  // KB and 256-byte chunks per block
        bool sparse = false;
        u32x4 blk[kQ] = {};
        auto load_blk = [&](uint32_t c0) __attribute__((always_inline)) {
#pragma unroll
            for (uint32_t i = 0; i < kQ; ++i) blk[i] = buf_load4(rin, 256 * c0 + 16 * (kQ * lane + i));
        };
        for (uint32_t ci = 0;;) {
            const bool more = ci < nch && !fgk.bad;
            uint32_t full = 0;
            if (kSparseOn && more && sparse) {
                if (np + 63 > kSymWords * 4) {
                    full = 1;  // room for a block's symbols first
                } else {
                    prio.at(ci, nch);
                    HC_PROF_BEGIN();
                    const uint32_t r = rle_block<kSrc, kQ>(blk, cy, sb_w, np, fgk.T.scratch, lane);
                    HC_PROF_END(4);
                    if (r != kDense) {
                        np = r;
                        ci += kBC;
                        full = np + 63 > kSymWords * 4 ? 1u : 0u;
                    }
                    if (r != kDense && ci + kBC < nch) {
                        load_blk(ci);
                    } else {  // a dense block or the last chunks: 256-byte chunks from ci
                        sparse = false;
                        next = buf_load(rin, 256 * ci + lane * 4);
                        ioff = 256 * ci + 256;
                    }
                }
            } else if (more) {
                const uint32_t m = ci + 1 < nch ? 256u : (uint32_t)(n - 256ull * ci);
                if (!redo) {
                    prio.at(ci, nch);
                    chunk = next;
                    if constexpr (kWin) {
                        if (ioff >= window) {  // slide the input window up to the next chunk
                            const uint64_t at = 256ull * (ci + 1);
                            rin = make_rsrc(bt.in + uni64(bt.in_offs[sid]) + at,
                                            (uint32_t)min((n - min(n, at) + 3u) & ~3ull, (uint64_t)kMaxBufBytes));
                            ioff = 0;
                        }
                        if ((sink.wout - sink.wbase) * 4ull >= window) sink.rebase(bt.out + out_off, cap);
                        next = buf_load(rin, ioff + lane * 4);  // out of range past the end: reads 0
                    } else {
                        next = buf_load(rin, ioff + lane * 4);
                    }
                    ioff += 256;
                }
                if (kSrc == SRC_SYMBOLS) {  // a ready symbol stream (adaptive path)
                    fgk.T.syms[lane] = chunk;
                    __builtin_amdgcn_wave_barrier();
                    np = m;
                    full = 1;  // coded at once
                } else {
                    // transform.cpp:220-229 (diff) + 241-279 (MNP-5 RLE), lane-parallel; symbols
                    // gather in syms[] (windowed streams: coded per chunk)
                    HC_PROF_BEGIN();
                    const uint32_t np0 = np;
                    uint32_t slanes = 64;
                    np = rle_chunk<kSrc>(chunk, m, ci + 1 == nch ? 1u : 0u, cy, sb_w, np, kWin ? 342u : kSymWords * 4,
                                         fgk.scr32(), lane, full, slanes);
                    HC_PROF_END(4);
                    if (kSparseOn && !full && slanes <= kSparseEnter && ci + 1 + kBC < nch) {
                        sparse = true;  // the block at ci + 1 (the chunk loaded ahead is dropped)
                        load_blk(ci + 1);
                    }
                    if (kWin) {
                        full = !full;  // code this chunk's symbols now (the chunk itself always fits)
                        redo = false;
                    } else {
                        redo = full != 0;
                        // code them now, too, when a next chunk like this one would not fit (a
                        // photo's chunk fills half the buffer: no chunk runs twice)
                        full |= np + (np - np0) > kSymWords * 4 ? 1u : 0u;
                    }
                }
                if (!redo) ++ci;
            }
            if (full || (!more && np)) {  // the serial FGK pass over the pending symbols
                if constexpr (kTab) code_all_tab(np);
                else if constexpr (kW <= 1 && HC_ENC_BATCH) {
#ifdef HC_PROF_PASS  // (diagnostic: region 3 times the whole batch pass instead of the record packing)
                    HC_PROF_BEGIN();
                    code_all_batch(np);
                    HC_PROF_END(3);
#else
                    code_all_batch(np);
#endif
                }
                else code_all(np);
                nsym += np;
                np = 0;
            }
            if (!more) break;
        }
    };
    if (n + 512 <= window && cap <= window) chunks(std::false_type{});
    else chunks(std::true_type{});

    const uint64_t total = sink.finish();
    const uint32_t st = fgk.bad ? (uint32_t)HC_ERR_DEVICE : (total <= cap ? 0u : (uint32_t)HC_ERR_CAPACITY);
    // headers.cpp:110-116: u64 little-endian symbol count in words 0-1 (stored after every
    // payload word by program order)
    buf_store(make_rsrc(bt.out + out_off, (uint32_t)min(cap, (uint64_t)8)), lane < 2 ? lane * 4 : kDrop,
              lane ? (uint32_t)(nsym >> 32) : (uint32_t)nsym);
    if (lane == 0) {
        bt.out_lens[sid] = fgk.bad ? 0 : total;
        bt.status[sid] = (int32_t)st;
    }
    trace_wave(sid, t0, lane);
    prof_store(sid, t0, pacc + fgk.pacc, lane);
}

// --------------------------------------------------------------------------- the decoder --

// MSB-first reader over a stream's bytes; words come from a 64-word VGPR chunk, the next chunk
// already loading (its wait falls ~64 refills later).
struct BitSource {
    rsrc_t rs;       // window of the stream at byte ibase
    uint64_t ibase;
    uint32_t lane;
    uint32_t cbase;  // byte offset of chunk lane 0 in the window
    uint32_t chunk;  // big-endian words (byte-swapped once per load, on the lanes)
    uint32_t nxt;    // the following 256 bytes as loaded
    uint32_t ridx;
    uint64_t win;  // upcoming bits, MSB-aligned
    uint32_t nwin; // valid bits in win

    __device__ __forceinline__ void next_word()
    {
        if (++ridx == 64) {
            cbase += 256;
            chunk = __builtin_bswap32(nxt);
            nxt = buf_load(rs, cbase + 256 + lane * 4);
            ridx = 0;
        }
    }
    // push the next 32 bits (needs nwin <= 32)
    __device__ __forceinline__ void refill()
    {
        const uint32_t w = lane_read(chunk, ridx);
        win |= (uint64_t)w << (32 - nwin);
        nwin += 32;
        next_word();
    }
    __device__ __forceinline__ uint32_t bit()
    {
        if (nwin == 0) refill();
        const uint32_t b = (uint32_t)(win >> 63);
        win <<= 1;
        --nwin;
        return b;
    }
    __device__ __forceinline__ uint32_t bits8()
    {
        if (nwin < 8) refill();
        const uint32_t b = (uint32_t)(win >> 56);
        win <<= 8;
        nwin -= 8;
        return b;
    }
};

// ------------------------------------------------------- RLE + diff revert (decoder) ------

// transform.cpp:137-159 (RLE revert) then 231-239 (diff revert) for one block of <= 256
// symbols, all lanes at once (model and derivation: tests/revert_block_model.py). The serial
// revert is a 4-state machine on the run counter r: in state 3 a symbol is a count (it emits
// that many copies of the previous symbol, r -> 0), else a literal (r -> r+1 when it repeats the
// previous symbol and r is 1 or 2, otherwise r -> 1). A symbol's transition is one of two
// functions on {0..3}, a 4-byte table (byte x = f(x)), so a composition is one v_perm_b32; a
// wave scan of the compositions gives each symbol's state, scans of output lengths and diff
// sums give each lane's output offset and running byte. Literals write their byte; a lane holds
// at most one count (counts follow three equal literals, so they are >= 4 symbols apart), and
// each count's run (an arithmetic sequence mod 256 with the diff model, a constant without)
// is written by the whole wave, 64 bytes per store.
struct RevCarry {
    uint32_t r;     // machine state after the last symbol
    uint32_t last;  // last symbol
    uint32_t prev;  // last output byte (diff model)
};

constexpr uint32_t kFeq = 1u | 2u << 8 | 3u << 16;  // r: 0->1 1->2 2->3 3->0
constexpr uint32_t kFne = 1u | 1u << 8 | 1u << 16;  // r: 0->1 1->1 2->1 3->0
constexpr uint32_t kFid = 0u | 1u << 8 | 2u << 16 | 3u << 24;

__device__ __forceinline__ uint32_t fsm_compose(uint32_t g, uint32_t f)  // x -> g(f(x))
{
    return __builtin_amdgcn_perm(0u, g, f);  // byte x = byte f(x) of g
}
__device__ __forceinline__ uint32_t fsm_apply(uint32_t f, uint32_t r) { return (f >> (8 * r)) & 255u; }

// lane l holds symbols 4l..4l+3 (m valid); bytes go to the stream's output at pos onwards (the
// buffer range check drops what is past the capacity); returns the bytes produced
__device__ __forceinline__ uint32_t revert_block(uint32_t x4, uint32_t m, RevCarry &cy, uint32_t dmask,
                                                 rsrc_t rs, uint32_t pos, uint32_t *row, uint32_t lane)
{
    const uint32_t xp = (x4 << 8) | (wave_shr1(x4, cy.last << 24) >> 24);  // previous symbols
    const uint32_t i0 = lane * 4;
    uint32_t f[4], F = kFid;
    for (uint32_t b = 0; b < 4; ++b) {
        f[b] = i0 + b < m ? (byte_of(x4, b) == byte_of(xp, b) ? kFeq : kFne) : kFid;
        F = fsm_compose(f[b], F);
    }
    // inclusive scan, lanes 0..l applied in order: DPP row shifts, then row broadcasts 15 and 31;
    // lanes without a source keep the identity
    uint32_t inc = F;
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x111, 0xF, 0xF, false));  // row_shr:1
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x112, 0xF, 0xF, false));  // row_shr:2
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x114, 0xF, 0xF, false));  // row_shr:4
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x118, 0xF, 0xF, false));  // row_shr:8
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x142, 0xA, 0xF, false));  // row_bcast:15
    inc = fsm_compose(inc, __builtin_amdgcn_update_dpp(kFid, inc, 0x143, 0xC, 0xF, false));  // row_bcast:31
    uint32_t r = fsm_apply(wave_shr1(inc, kFid), cy.r);
    uint32_t len[4], c[4], tot = 0, ds = 0, cnt_b = 4;  // cnt_b: the lane's count symbol (4: none)
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t sb = byte_of(x4, b), pb = byte_of(xp, b);
        const bool valid = i0 + b < m;
        const bool cnt = r == 3;
        len[b] = valid ? (cnt ? sb : 1u) : 0u;
        c[b] = cnt ? pb : sb;
        ds += valid ? (cnt ? sb * pb : sb) : 0u;
        tot += len[b];
        cnt_b = valid && cnt ? b : cnt_b;
        r = fsm_apply(f[b], r);
    }
    // exclusive scans of (length, diff sum mod 256), packed: both halves stay below 2^16
    const uint32_t mine = tot | ((ds & 255u) << 16);
    const uint32_t acc = RecSink::scan_add(mine);
    const uint32_t exc = acc - mine;
    uint32_t prev = (cy.prev + (exc >> 16)) & 255u;
    uint32_t o = pos + (exc & 0xFFFFu);
    // literals; the count only records its run: output offset, length | base << 8 | step << 16
    // (run byte j = base + step * (j + 1); base = the byte before it, or the repeated byte
    // itself with step 0 without the diff model)
    uint32_t ro = 0, rlen = 0;
    for (uint32_t b = 0; b < 4; ++b) {
        if (b == cnt_b) {
            rlen = dmask ? (len[b] | prev << 8 | c[b] << 16) : (len[b] | c[b] << 8);
            ro = o;
            prev = dmask ? (prev + len[b] * c[b]) & 255u : (len[b] ? c[b] : prev);
        } else {
            prev = ((prev & dmask) + c[b]) & 255u;
            buf_store8(rs, len[b] ? o : kDrop, prev);
        }
        o += len[b];
    }
    // the runs (run byte j = v1 + st1 * j), 16 at a time, four lanes each: a run's 16-byte units
    // (aligned in memory) go four per store, 64 contiguous bytes a run, then the <= 15 + 15 bytes
    // before and after them four per store -- grad -c -m (~54 runs of ~255 bytes per block) takes
    // 4 groups of ~4 + ~8 steps instead of a pass of the whole wave per run and 64 bytes
    // (measured: grad decode 1.30 -> 1.17 ms, C5 383 -> 380, noise 164.5 -> 161; without the run
    // stores at all 0.92 ms; one run per lane, 16-byte units scattered over 64 runs per store,
    // 1.36 ms; whole dwords run by run 1.30 ms: the run loop's instructions, not its stores). A block whose runs reach past the
    // output window (a capacity error) goes run by run, byte by byte, so every byte before the
    // end lands.
    const uint32_t n = rlen & 255u;
    const uint32_t st1 = dmask ? rlen >> 16 : 0u, v1 = (((rlen >> 8) & 255u) + st1) & 255u;
    const uint64_t rm = ballot(n != 0);
    if (rm && !ballot(ro + n > rs.bytes)) {
        // the lanes that hold a run, in order: row[k] = the k-th one
        if (n) row[__builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u))] = lane;
        __builtin_amdgcn_wave_barrier();
        const uint32_t nr = (uint32_t)__builtin_popcountll(rm), q = lane & 3u;
        const uint32_t spec = n | st1 << 8 | v1 << 16;
        constexpr uint32_t kL7 = 0x7F7F7F7Fu, kH = 0x80808080u;
        auto add8 = [&](uint32_t a, uint32_t b) __attribute__((always_inline)) {
            return ((a & kL7) + (b & kL7)) ^ ((a ^ b) & kH);
        };
        for (uint32_t g = 0; g < nr; g += 16) {
            const uint32_t r = g + (lane >> 2);
            const uint32_t src = row[r < nr ? r : 0u] * 4;
            // (both permutes on every lane: a source lane outside the exec mask would give 0)
            const uint32_t gs0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)spec);
            const uint32_t go = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)ro);
            const uint32_t gs = r < nr ? gs0 : 0u;
            const uint32_t gn = gs & 255u, gst = (gs >> 8) & 255u, gv = gs >> 16;
            const uint32_t hb = min((0u - ((uint32_t)rs.base + go)) & 15u, gn);  // bytes before the units
            const uint32_t nu = (gn - hb) >> 4, eb = gn - 16 * nu;                // units; edge bytes
            // bytes j0 .. j0 + 15: a splat of byte j0 plus (0, s, 2 s, 3 s), then + 4 s per byte for
            // each next dword (bytewise adds without carries)
            const uint32_t P = ((gst & 255u) << 8 | ((2 * gst) & 255u) << 16 | ((3 * gst) & 255u) << 24);
            const uint32_t S4 = __builtin_amdgcn_perm(0u, 4u * gst, 0u);
            uint32_t u = q, x = gv + gst * (hb + 16 * q), o = go + hb + 16 * q;
            while (ballot(u < nu)) {
                u32x4 w;
                w[0] = add8(__builtin_amdgcn_perm(0u, x, 0u), P);
                w[1] = add8(w[0], S4);
                w[2] = add8(w[1], S4);
                w[3] = add8(w[2], S4);
                buf_store4(rs, u < nu ? o : kDrop, w);
                u += 4;
                x += 64u * gst;
                o += 64u;
            }
            for (uint32_t e = q; ballot(e < eb); e += 4) {
                const uint32_t j = e < hb ? e : e + 16 * nu;
                buf_store8(rs, e < eb ? go + j : kDrop, gv + gst * j);
            }
        }
        __builtin_amdgcn_wave_barrier();
    } else {
        for (uint64_t runs = ballot(n != 0); runs; runs &= runs - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(runs);
            const uint32_t at = lane_read(ro, l), rn = lane_read(n, l), rv = lane_read(v1, l), rs1 = lane_read(st1, l);
            for (uint32_t j0 = 0; j0 < rn; j0 += 64) {
                const uint32_t j = j0 + lane;
                buf_store8(rs, j < rn ? at + j : kDrop, rv + rs1 * j);
            }
        }
    }
    const uint32_t all = lane_read(acc, 63);
    cy.r = fsm_apply(lane_read(inc, 63), cy.r);
    cy.last = byte_of(lane_read(x4, (m - 1) >> 2), (m - 1) & 3u);
    cy.prev = (cy.prev + (all >> 16)) & 255u;
    return all & 0xFFFFu;
}

// One stream's decoder (huffman.cpp:60-93 + transform.cpp:386-406 per symbol, then the RLE and
// diff revert of transform.cpp:137-159 / 231-239 per 256-symbol block; header main.cpp:90-104).
// decode_kernel runs one per wavefront.
// The small-alphabet launch (decode_kernel<0, .., true>, Dec::decode_small) takes the narrow
// streams whose payload averages under 2.5 bits per symbol -- the header's count and the
// stream's length, so the decoder needs no sample of its own (grad -c -m: 1.7; photo -c -m:
// 3.3-3.6; noise, -c photos: ~8). mode (hc_debug_set_dec_small): 0 by the rate, 1 every narrow
// stream, 2 none. Either launch decodes any stream exactly; the rate only picks the faster.
__device__ __forceinline__ bool dec_small_stream(uint64_t count, uint64_t bits, uint32_t mode)
{
    if (mode) return mode == 1;
    return count != 0 && bits * 2 < count * 5;
}

template <int kW, int kDst, bool kSmall = false>
struct Dec {
    // symbol indices: 32-bit below 2^32 symbols (narrow / wide), 64-bit for the huge layout
    using Idx = std::conditional_t<kW == 2, uint64_t, uint32_t>;
    Fgk<kW, true, false, kSmall> fgk;
    BitSource in;
    uint32_t lane, sid, st, dmask;
    uint64_t len, cap, payload_bits;
    uint64_t obase;  // output window at byte obase (slides with the output, like the input's)
    uint64_t pos;    // output bytes produced
    rsrc_t rout;
    RevCarry rc;
    uint8_t *sbuf;  // this block's symbols (LDS)
    Idx n;
    uint32_t bsym = 0, btry = 0;  // this block's batch symbols and batches
    Prio<Idx> prio;
    bool batch_on = true;          // the next block runs batches
    uint64_t pacc = 0;  // HC_PROF regions

    __device__ __forceinline__ Dec(Tree<kW, true, false, kSmall> &t, uint32_t l) : fgk(t, l), lane(l) {}

    // the stream's header; false: nothing to decode here (its error status is written, or another
    // tree layout's launch owns it)
    __device__ __forceinline__ bool open(const Batch &bt, uint32_t s)
    {
        sid = s;
        const uint64_t in_off = uni64(bt.in_offs[sid]);
        len = uni64(bt.in_lens[sid]);
        cap = uni64(bt.out_caps[sid]);
        const uint32_t len32 = (uint32_t)min(len, (uint64_t)kMaxBufBytes);
        const rsrc_t rin = make_rsrc(bt.in + in_off, (len32 + 3u) & ~3u);
        const uint32_t hdr = buf_load(rin, lane * 4);  // words 0..63 of the stream
        st = 0;
        uint64_t count = 0;
        uint32_t flags = 0;
        if (len < 9) {
            st = HC_ERR_HEADER;  // main.cpp:99-104
        } else {
            count = (uint64_t)lane_read(hdr, 0) | ((uint64_t)lane_read(hdr, 1) << 32);
            flags = lane_read(hdr, 2) & 255u;
            const uint64_t avail = (len - 9) * 8;
            // the first symbol costs >= 8 bits and each later one >= 1: a larger count cannot
            // decode, and the reference ends such a stream with status 9 (transform.cpp:394-398)
            if (count > (avail >= 8 ? avail - 7 : 0)) st = HC_ERR_HUFFMAN;
            else if (kDst == DST_RAW && (flags & 0x40u)) st = HC_ERR_UNSUPPORTED;
        }
        if (st == 0 && tree_kind(count, bt.min_tree) != (uint32_t)kW) return false;  // another layout's launch owns it
        // narrow streams under 2.5 payload bits per symbol go to the small-alphabet launch
        // (dec_small_stream), the rest to the regular one
        if (st == 0 && kW == 0 && dec_small_stream(count, (len - 9) * 8, bt.dec_small) != kSmall) return false;
        if (st != 0) {
            if (kW == 0 && !kSmall && lane == 0) {
                bt.status[sid] = (int32_t)st;
                bt.out_lens[sid] = 0;
            }
            return false;
        }
        in.rs = rin;
        in.ibase = 0;
        in.lane = lane;
        in.cbase = 0;
        in.chunk = __builtin_bswap32(hdr);
        in.nxt = buf_load(rin, 256 + lane * 4);
        in.ridx = 2;
        in.win = 0;
        in.nwin = 0;
        in.refill();  // word 2: flags byte + first payload bits
        in.win <<= 8;
        in.nwin -= 8;
        rout = make_rsrc(bt.out + uni64(bt.out_offs[sid]), (uint32_t)min(cap, (uint64_t)kMaxBufBytes));
        obase = 0;
        pos = 0;
        dmask = kDst == DST_RAW && (flags & 0x80u) ? 255u : 0u;  // diff model
        rc = {0, 0, 0};
        sbuf = reinterpret_cast<uint8_t *>(fgk.T.syms);
        n = (Idx)count;
        payload_bits = (len - 9) * 8;
        return true;
    }
    // input and output fit one buffer window (every batch stream): no window bookkeeping
    __device__ __forceinline__ bool one_window() const
    {
        const uint32_t window = window_bytes();
        return len + 512 <= window && cap <= window;
    }
    // bits read from the stream = words pushed into the window * 32 - bits still in it; the
    // payload starts at bit 72. A stream that ends early decodes zero bits past its end (the
    // range check); the reference stops there with status 9 (transform.cpp:394-398), which is
    // what close() reports.
    __device__ __forceinline__ uint64_t consumed() const { return ((in.ibase + in.cbase) / 4 + in.ridx) * 32 - in.nwin - 72; }
    __device__ __forceinline__ bool stopped() const { return fgk.bad || consumed() > payload_bits + 64; }
    // a block's symbols end at i1
    __device__ __forceinline__ Idx block_end(Idx i0) const
    {
        if constexpr (kW == 2) return n - i0 < 256 ? n : i0 + 256;
        else return min(n, i0 + 256);
    }

    template <bool kWin>
    __device__ __forceinline__ void block_start(const Batch &bt, Idx i0)
    {
        if constexpr (kWin) {
            const uint32_t window = window_bytes();
            if (in.cbase >= window) {  // slide the input window to the current chunk (a block of
                in.ibase += in.cbase;  // 256 symbols reads < 2 KB, so offsets stay below 2^31)
                in.cbase = 0;
                const uint64_t l = uni64(bt.in_lens[sid]);
                in.rs = make_rsrc(bt.in + uni64(bt.in_offs[sid]) + in.ibase,
                                  (uint32_t)min((l - min(l, in.ibase) + 3u) & ~3ull, (uint64_t)kMaxBufBytes));
            }
            if (pos - obase >= window) {  // and the output window to the next byte
                obase = pos;
                rout = make_rsrc(bt.out + uni64(bt.out_offs[sid]) + obase,
                                 obase < cap ? (uint32_t)min(cap - obase, (uint64_t)kMaxBufBytes) : 0u);
            }
        }
        prio.at(i0, n);
    }

    // symbol i - 1 (of the block at i0) left the hot loop with its leaf entry's position x and
    // depth d, the body b read at x, the root path pv and the first level k whose leader test
    // failed (the window stands d bits into its code): finish it
    __device__ __forceinline__ void finish_symbol(uint32_t b, uint32_t pv, uint32_t k, uint32_t d, uint32_t x, Idx i, Idx i0)
    {
        if (!(b & (kInner | kNyt))) {  // a leaf whose update reported level k: walk from there
            HC_PROF_BEGIN();
            fgk.walk(lane_read(pv, k), pv);
            HC_PROF_END(1);
            return;
        }
        // nothing was stored for it
        uint32_t sym = 0;
        bool deep = false;  // a code longer than the cache's 9 levels: a rare symbol
        HC_PROF_BEGIN();
        if (b & kInner) {
            // the code is longer than the tables reach, or they stopped short (a leaf that
            // split since): descend bit by bit, top-down first (depth j at lane 64-j),
            // then turned bottom-up
            uint32_t depth = d;
            fgk.stale += depth < 8 ? 1u : 0u;
            if (fgk.stale >= kRefresh) fgk.from = 0;
            // levels 1..8 of the prefix, lane 64 - j <- level j (lane 8 - j of the path read)
            uint32_t pt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - 56) & 63u) * 4), (int)pv);
            // the position and its body stay in VGPRs (wave-uniform): per level the child address,
            // one read, a select into lane 63 - depth (a scalar bit mask) and the inner test by a
            // ballot -- no hop through the scalar unit per level (~22 -> ~13 instructions). The
            // tree is the kernel's own (input bits only choose the child), and the depth bound ends
            // the walk down on any inconsistency.
            // The window's bits are taken straight from a copy of it; the refill (and the 63-level
            // bound) is tested once per level against lim, the depth the bits in the window reach.
            const uint32_t bbase = lds_off16(&fgk.T.body[0]);
            uint32_t xv = vreg(x), bv = vreg(b);
            if (in.nwin <= 32) in.refill();
            uint64_t w = in.win;
            uint32_t d0 = depth, lim = min(depth + in.nwin, 63u);
#pragma unroll 1
            for (;;) {
                uint64_t inner;
#pragma unroll 1
                do {
                    const uint32_t bit = (uint32_t)(w >> 63);
                    w <<= 1;
                    xv = ((bv << 1) & 0x1FEu) | bit;  // child pair * 2 + bit
                    pt = sel(1ull << (63 - depth), xv, pt);
                    ++depth;
                    bv = opaque(*(const lds_u16 *)(size_t)(bbase + 2 * xv));
                    // go on while the body is inner and the window has bits: one compare
                    // (inner bit > stop) the branch takes as it is
                    uint32_t stop = (lim - depth - 1u) >> 31;  // depth >= lim (both < 64)
                    asm("" : "+s"(stop));  // kept an integer (a compare would go through a select)
                    inner = ballot(((bv >> 8) & 1u) > stop);
                } while (inner);
                if (!ballot(bv & kInner) || depth >= 63) break;
                // the window is used up (rare): its next word
                in.win = w;
                in.nwin -= depth - d0;  // 0
                in.refill();
                w = in.win;
                d0 = depth;
                lim = min(depth + in.nwin, 63u);
            }
            in.win = w;
            in.nwin -= depth - d0;
            x = uni(xv);
            b = uni(bv);
            if (depth > 62) fgk.bad = 1;  // beyond the lanes (needs > 2^32 symbols)
            deep = depth > kInsertDepth;
            pv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((64 - depth + lane) & 63u) * 4), (int)pt);
            pv = lane < depth ? pv : kRoot;
            sym = b & 255u;
        }
        if (b & kNyt) {  // the new leaf below the NYT becomes level 0
            sym = in.bits8();
            // huffman.cpp:95-111 splits only for a symbol without a leaf; a corrupted stream
            // can name a known one, whose own leaf is then updated
            const uint32_t known = fgk.find_leaf(sym);
            if (known == 0xFFFFFFFFu) {
                x = uni(fgk.split(sym));
                pv = __shfl_up(pv, 1, 64);
                pv = lane == 0 ? x : pv;
            } else {
                fgk.chase(known, pv);
            }
        }
        HC_PROF_END(2);
        if (!(b & kInner)) {
            HC_PROF_BEGIN();
            // a rare symbol's leaf nearly always ties with the next position (9 in 10 on
            // the slot-form model): walk from the leaf at once
            if (deep) fgk.walk(lane_read(pv, 0), pv);
            else fgk.update_path(pv);
            HC_PROF_END(3);
        }
        sbuf[i - 1 - i0] = (uint8_t)sym;
    }

#if HC_DEC_BATCH
    // Batched hot path (narrow and wide layouts; model: tests/fgk_batch_model.py decode_batch).
    // Between swaps and splits the tree's shape -- and with it every code -- is fixed, and the
    // update of a symbol whose levels all pass the leader test only adds 1 along its root path.
    // So up to kB symbols are decoded in a row from the level tables alone (lane 9 j + l: level
    // 8 - l of symbol j's lookup; one read per symbol, the window shifted by the depths read)
    // and tested at once:
    //  1. every batch symbol's path positions (each once: the lanes whose entry stops at their
    //     own level; the root once per symbol) get their increment tentatively, one LDS add,
    //     the words of the next positions having been read before;
    //  2. a level fails when that next word is below the position's word after the adds: the
    //     one-symbol loop's test with every batch symbol through the position counted as
    //     earlier (c0 at its largest) and none through the next one (c1 = 0), so it can report
    //     a level falsely, never pass one that fails (the model: 2 % more symbols decoded alone
    //     on a photo than with exact counts);
    //  3. the increments of the first failing symbol and the ones after it are taken back. The
    //     symbols before it are decoded; it -- or the first symbol whose entry is not a leaf (a
    //     code longer than the tables, or the NYT) -- goes to the one-symbol step.
    // Returns whether the batch took every symbol the window and the block allowed (otherwise the
    // one-symbol step takes the next one).
    __device__ __forceinline__ bool decode_batch(Idx i0, Idx &i, Idx i1)
    {
        constexpr uint32_t kG = 9, kB = HC_DEC_BATCH;  // lanes per symbol (levels 8..0), symbols
        static_assert(kB * kG <= 63, "batch lanes");
        const uint32_t bj = lane < kB * kG ? lane / kG : 7u;  // the lane's symbol (7: idle)
        const uint32_t bl = lane < kB * kG ? lane % kG : 8u;  // its level: 8 - bl
        const uint32_t bsh = 24 + min(bl, 7u);
        const uint32_t bvb = lds_off16(&fgk.T.lvl[0]) + 2 * (bl < 8 ? (256u >> bl) - 2 : 0xFFFFFFFEu);
        const uint32_t l8 = lds_off16(&fgk.T.lvl[254]);  // level 8
        const uint64_t w0 = in.win;
        const uint32_t n0 = in.nwin;  // >= 33: symbols 0..3 always fit
        // lane o: the depth of a code that starts o bits into the window (its level-8 entry);
        // the chain of symbol starts then runs on registers: S_j+1 = S_j + depth(S_j). sv lane j:
        // the bits before symbol j.
        const uint32_t dep = opaque(*(const lds_u16 *)(size_t)(l8 + 2 * (uint32_t)((w0 << lane) >> 56))) >> 10;
#if HC_DEC_EXIT8
        // a first code of 8 bits or more (most of them on a flat alphabet, e.g. noise, where codes
        // are longer than the tables) goes to the one-symbol step at once
        if (lane_read(dep, 0) >= 8) {
            ++btry;
            return false;
        }
#endif
        // (measured and dropped: the chain by pointer doubling -- lane o's next start o + depth(o),
        // composed by permutes, lane j applying them by the bits of j: 11 VALU + 4 LDS instead of
        // ~16 VALU + 7 SALU, but its dependent permutes made C5 decode +0.8 %)
        uint32_t S = 0, sv = 0;
        const uint32_t bj4 = bj * 4;
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            sv = writelane(sv, S, j);
            S += lane_read(dep, S);
        }
        sv = writelane(sv, S, kB);
        // each lane's own symbol's start: one permute (measured: C5 decode -5.5 % against a select
        // per symbol in the chain, 14 VALU instructions per step)
        const uint32_t sg = (uint32_t)__builtin_amdgcn_ds_bpermute((int)bj4, (int)sv);
        // symbols whose code lies inside the window (lane j + 1: the bits up to symbol j's end)
        const uint32_t nval = __builtin_popcountll(ballot(sv <= n0) & (((1ull << kB) - 1) << 1));
        const uint32_t jmax = min(nval, (uint32_t)(i1 - i));
        // every symbol's whole root path at once, each group on its own window
        const uint32_t ent = opaque(*(const lds_u16 *)(size_t)(bvb + (((uint32_t)((w0 << sg) >> 32) >> bsh) << 1)));
        const uint32_t pos = ent & 1023u;
        // the lanes that add: each path position once (the entry stops at the lane's own level),
        // symbols inside the window and the block
        const uint64_t actm = ballot((ent >> 10) == 8 - bl) & groups9(jmax);
        constexpr uint32_t kI = kW ? 1u : 1024u;
        const uint32_t wa = lds_off(&fgk.T.wt[0]) + 4 * pos;
        const uint32_t scr = lds_off(fgk.scr32());
        // a leaf's body is its symbol; bit 15: inner or NYT (read with the weights: a symbol whose
        // entry is no leaf has its increments taken back like a failing one)
        const uint32_t b = opaque(*(const lds_u16 *)(size_t)(lds_off16(&fgk.T.body[0]) + 2 * pos));
        const uint32_t w1 = *(const lds_u32 *)(size_t)(wa + 4);
        __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(actm, wa, scr), kI, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t wn = *(const lds_u32 *)(size_t)wa;
        constexpr uint64_t kLeafLanes = 0x0040201008040201ull & ((1ull << (kB * kG)) - 1);
        // (ff1 of no lane: 0xFFFFFFFF, above every batch)
        const uint32_t jn = ff1(ballot(b & kNotLeaf) & kLeafLanes) / kG;
        uint64_t ft = ballot(w1 < wn) & actm;
        uint32_t jf = min(min(ff1(ft) / kG, jn), jmax);
        if (jf < jmax) {
            __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(actm & ~groups9(jf), wa, scr), 0u - kI,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#if HC_BATCH_RETRY
            // 4. retest in place when the failure of symbol jf (a leaf) may be false, as the
            // encoder's code_all_batch does: the symbols before it committed, the words of its a
            // and a + 1 hold the earlier symbols' exact counts
            uint32_t j0 = 0;
            while (jf > j0 && jf < jn) {
                const uint64_t gl = groups9(jf);
#if HC_BATCH_RETRY == 1
                const uint32_t fa = lane_read(pos, ff1(ft));
                if (!((ballot(pos == fa + 1) & gl) | (ballot(pos == fa) & actm & ~groups9(jf + 1)))) {
                    HC_CNT(4);
                    break;
                }
#endif
                HC_CNT(3);
                const uint64_t am2 = actm & ~gl;  // symbols jf..
                const uint32_t w1r = *(const lds_u32 *)(size_t)(wa + 4);
                __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(am2, wa, scr), kI, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WAVEFRONT);
                const uint32_t wnr = *(const lds_u32 *)(size_t)wa;
                ft = ballot(w1r < wnr) & am2;
                j0 = jf;
                jf = min(min(ff1(ft) / kG, jn), jmax);
                if (jf > j0) HC_CNT(6);
                if (jf == jmax) break;
                __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel(actm & ~groups9(jf), wa, scr), 0u - kI,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
#endif
        }
        const uint32_t sb0 = (uint32_t)(size_t)(lds_u8 *)sbuf + (uint32_t)(i - i0);
        *(lds_u8 *)(size_t)sel(kLeafLanes & groups9(jf), sb0 + bj, scr) = (uint8_t)b;
        __builtin_amdgcn_wave_barrier();
        HC_CNT(1);
        if (jf < jmax) HC_CNT(2);
        if (jf == jn && jf < jmax) HC_CNT(5);
        const uint32_t sj = lane_read(sv, jf);
        in.win = w0 << sj;
        in.nwin = n0 - sj;
        i += jf;
        bsym += jf;
        ++btry;
        return jf == jmax;
    }

    // Small alphabets (the small-alphabet launch, narrow layout, while at most 16 symbols are
    // seen: every position >= kSmallNyt; the encoder's small steps in code_all_batch, whose
    // output this reads back). Up to 15 symbols of depth <= 4 per step, four lanes each (lane
    // 4 j + l: level 4 - l of symbol j's lookup in the level tables); the chain of symbol starts
    // from the level-4 depths at every bit offset (<= 4 bits a symbol: 60 bits at most). The
    // leader tests are exact, as in the encoder: every path position ORs its symbol's bit into a
    // membership mark (smark), and symbol j's test at position a reads the pre-step words of a
    // and a + 1 and the marks of both: with c0 / c1 the earlier symbols through a / a + 1 (c1 = j
    // at the root) the level passes iff weight(a + 1) + c1 >= weight(a) + c0 + 1. The first
    // symbol with a failing level, or whose level-4 entry is no leaf (deeper than 4, or the
    // NYT), ends the step: the ones before it commit with one add (the root by lane 63), it goes
    // to the one-symbol step. Returns whether the step took every symbol the window and the
    // block allowed.
    __device__ __forceinline__ bool decode_small(Idx i0, Idx &i, Idx i1)
    {
        static_assert(kW == 0 && kSmall, "the small-alphabet launch: narrow layout");
        constexpr uint32_t kSG = kSmallG, kSK = kSmallK;
        constexpr uint64_t kL63 = 1ull << 63;
        // (the lane index opaque: these per-lane values are made here, not hoisted beside the
        // regular batch's)
        const uint32_t ln = vreg(lane);
        const uint32_t g = ln < kSK * kSG ? ln >> 2 : kSK;  // the lane's symbol (kSK: idle)
        const uint32_t bl = ln & 3u;                        // its level: 4 - bl
        const uint32_t bvb = lds_off16(&fgk.T.lvl[0]) + 2 * ((16u >> bl) - 2);
        const uint32_t l4 = lds_off16(&fgk.T.lvl[14]);  // level 4
        const uint32_t sscb = lds_off(&fgk.T.scratch[0]) + 4 * ln;
        const uint32_t mkb = lds_off(&fgk.T.smark[0]);
        const uint64_t w0 = in.win;
        const uint32_t n0 = in.nwin;  // >= 33: symbols 0..7 always fit
        // lane o: the depth of a code that starts o bits into the window (4 when deeper)
        const uint32_t dep = opaque(*(const lds_u16 *)(size_t)(l4 + 2 * (uint32_t)((w0 << ln) >> 60))) >> 10;
        // each lane's own code start by a select per chain step (measured: grad decode 1.172 ->
        // 1.158 ms against one permute after the chain, whose round trip the step waits for)
        uint32_t S = 0, sv = 0, sg = 0;
#pragma unroll
        for (uint32_t j = 0; j < kSK; ++j) {
            sv = writelane(sv, S, j);
            sg = g == j ? S : sg;
            S += lane_read(dep, S);
        }
        sv = writelane(sv, S, kSK);
        const uint32_t nval = __builtin_popcountll(ballot(sv <= n0) & (((1ull << kSK) - 1) << 1));
        const uint32_t jmax = min(nval, (uint32_t)(i1 - i));
        const uint32_t ent = opaque(*(const lds_u16 *)(size_t)(bvb + (((uint32_t)((w0 << sg) >> 32) >> (28 + bl)) << 1)));
        uint32_t pos = ent & 1023u;
        pos = sel(~0ull << (kSK * kSG), kRoot, pos);  // lane 63: the root
        const uint64_t gm = below_mask(kSG * jmax);
        // each path position once (the entry stops at the lane's own level)
        const uint64_t am = ballot((ent >> 10) == 4 - bl) & gm;
        const uint32_t wa = lds_off(&fgk.T.wt[0]) + 4 * pos;
        const uint32_t b = opaque(*(const lds_u16 *)(size_t)(lds_off16(&fgk.T.body[0]) + 2 * pos));
        constexpr uint64_t kLeafLanes = 0x0111111111111111ull;  // level 4: lanes 4 j
        const uint32_t jn = ff1(ballot(b & kNotLeaf) & kLeafLanes) >> 2;
        const uint32_t wl = *(const lds_u32 *)(size_t)wa, wh = *(const lds_u32 *)(size_t)(wa + 4);
        const uint32_t ma = pos - kSmallNyt, odd = ma & 1u;  // (pos >= 480 on the am lanes)
        const uint32_t mda = sel(am, mkb + 4 * (ma >> 1), sscb);
        __hip_atomic_fetch_or((uint32_t *)(lds_u32 *)(size_t)mda, (1u << g) << (odd << 4), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t mlo = *(const lds_u32 *)(size_t)mda;
        const uint32_t mhi = *(const lds_u32 *)(size_t)(mda + 4 * odd);
        const uint32_t c0 = (uint32_t)__builtin_popcount(__builtin_amdgcn_ubfe(mlo, odd << 4, g));
        const uint32_t c1 = pos + 1 == kRoot ? g : (uint32_t)__builtin_popcount(__builtin_amdgcn_ubfe(odd ? mhi : mlo, (odd ^ 1u) << 4, g));
        const uint64_t fm = ballot((wh >> 10) + c1 < (wl >> 10) + c0 + 1) & am;
        const uint32_t jf = min(min(ff1(fm) >> 2, jn), jmax);
        __hip_atomic_fetch_add((uint32_t *)(lds_u32 *)(size_t)sel((am & below_mask(kSG * jf)) | kL63, wa, sscb),
                               sel(kL63, jf << 10, 1u << 10), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        *(lds_u32 *)(size_t)mda = 0u;
        const uint32_t sb0 = (uint32_t)(size_t)(lds_u8 *)sbuf + (uint32_t)(i - i0);
        *(lds_u8 *)(size_t)sel(kLeafLanes & below_mask(kSG * jf), sb0 + g, sscb) = (uint8_t)b;
        __builtin_amdgcn_wave_barrier();
        HC_CNT(1);
        if (jf < jmax) HC_CNT(2);
        const uint32_t sj = lane_read(sv, jf);
        in.win = w0 << sj;
        in.nwin = n0 - sj;
        i += jf;
        bsym += jf;
        ++btry;
        return jf == jmax;
    }
#endif

    // symbols i .. i1 - 1 of the block at i0, one stream
    // kBat: batches first (narrow / wide layouts), the one-symbol step after each batch that
    // stops short; otherwise the one-symbol loop alone
    template <bool kBat = (kW <= 1)>
    __device__ __forceinline__ void decode(Idx i0, Idx &i, Idx i1)
    {
        while (i < i1) {
            // huffman.cpp:60-93: the code's first 8 bits index the level tables: level 8 gives
            // where the walk from the root stops (depth d <= 8), the levels above give the
            // positions the walk passes.
            if (fgk.from < 9) {
                HC_PROF_BEGIN();
                fgk.build_levels();
                HC_PROF_END(5);
            }
            if (in.nwin <= 32) in.refill();
#if HC_DEC_BATCH
            // batches, and the symbol that ends one alone (kOne: the one-symbol step takes one)
            constexpr bool kOne = kBat && kW <= 1;
            if constexpr (kOne) {
                HC_PROF_BEGIN();
                bool whole;
                if constexpr (kSmall) whole = fgk.nyt >= kSmallNyt ? decode_small(i0, i, i1) : decode_batch(i0, i, i1);
                else whole = decode_batch(i0, i, i1);
                HC_PROF_END(6);
                if (whole) continue;
                if (in.nwin <= 32) in.refill();
            }
#else
            constexpr bool kOne = false;
#endif
            // Hot loop: a leaf within the tables' reach whose update needs no walk. Once a
            // symbol's depth is known the next symbol's table entry is read, before this
            // symbol's update (the tables and body[] change only on the paths that leave the
            // loop, and the loop is re-entered after them). Anything else
            // (a longer code or a stale table: body inner; the NYT; a failed leader test) is
            // forced to fail at level 0 so nothing is stored, and is finished outside.
            // lane k reads level 8 - k's entry for the code's 8-bit prefix v, at
            // ((256 | v) >> k) - 2: levels >= d repeat the leaf's entry (position | depth d), so
            // lanes 0..8-d hold the leaf, lanes 9-d..7 its ancestors (level 8-k), lane 8 and up
            // the root pad (lvl_root). One read gives the depth (lane 0) and the whole root path
            // (duplicated lanes store the same word); it depends only on the window, so the next
            // code's read goes out as soon as this code's depth is known.
            // ((256 | v) >> k) - 2 = (v >> k) + (256 >> k) - 2, and v >> k = window bits 56 + k..63:
            // one per-lane shift of the window's high word and one per-lane base; lanes 8 and up
            // shift by 31 and land on lvl_root[-2 + 0/1] (both the root)
            const uint32_t vsh = 24 + min(lane, 7u);
            const uint32_t vbase = lds_off16(&fgk.T.lvl[0]) + 2 * (lane < 8 ? (256u >> lane) - 2 : 0xFFFFFFFEu);
            auto path_read = [&](uint64_t w) __attribute__((always_inline)) {
                return opaque(*(const lds_u16 *)(size_t)(vbase + ((uint32_t)(w >> 32) >> vsh) * 2));
            };
            uint32_t pr = path_read(in.win);
            const uint32_t bbase = lds_off16(&fgk.T.body[0]);
            uint32_t d, x, b, pv, k;
            // loop while no level failed (k = 0xFFFFFFFF) and symbols are left (left < 0):
            // both sign bits set, one scalar AND (after a batch: one symbol)
            int32_t left = kOne ? -1 : (int32_t)(i - i1);
            lds_u8 *so = (lds_u8 *)sbuf + (uint32_t)(i - i0);  // the symbol's byte (LDS address in a VGPR)
            // The leaf's body: every lane reads the body at its own path position; one row_newbcast DPP move gives
            // rows 0 its lane 0's (the leaf's), so the read needs no scalar address. Lanes 16 and up
            // (root padding) read lvl_root instead (kRoot: bit 15 clear, no force) and put their
            // copy of the symbol byte in the landing row, not the block.
            const uint32_t vbb = lane < 16 ? bbase : lds_off16(&fgk.T.lvl_root[0]) - 2 * kRoot;
            so += lane < 16 ? 0 : (uint32_t)((uint8_t *)fgk.T.scratch - sbuf);
            uint32_t e8;
            asm("" : "+v"(so));
            do {
                e8 = uni(pr);  // the leaf's entry
                d = e8 >> 10;
                pv = pr & 1023u;
                b = (uint32_t)__builtin_amdgcn_mov_dpp((int)opaque(*(const lds_u16 *)(size_t)(vbb + 2 * pv)), 0x150, 0xF, 0xF, false);
                in.win <<= d;
                in.nwin -= d;  // >= 25
                uint32_t prn;
                // a leaf's body is its symbol; inner / NYT (bit 15): force the failure
                const uint32_t force = (uint32_t)__builtin_amdgcn_sbfe((int)b, 15, 1);
                k = fgk.update_fast(pv, [&] { prn = path_read(in.win); }, force);  // the next code's
                *so++ = (uint8_t)b;  // the symbol (a leaf's body); rewritten when it leaves
                ++left;
                if (in.nwin <= 32) in.refill();
                pr = prn;
            } while ((int32_t)(k & (uint32_t)left) < 0);
            i = i0 + uni((uint32_t)(so - (lds_u8 *)sbuf));
            if (k == 0xFFFFFFFFu) continue;
            x = e8 & 1023u;
            // symbol i - 1 left the loop: the window stands d bits into its code
            finish_symbol(uni(b), pv, k, uni(d), uni(x), i, i0);
        }
    }

    // the block's symbols [i0, i1) leave: reverted to bytes (transform.cpp:137-159, 231-239) or
    // stored as they are (the adaptive path's symbol stream)
    __device__ __forceinline__ void close_block(Idx i0, Idx i1)
    {
        __builtin_amdgcn_wave_barrier();
        const uint32_t x4 = fgk.T.syms[lane];
        const uint32_t m = (uint32_t)(i1 - i0);
        if (kDst == DST_SYMBOLS) {
            for (uint32_t b = 0; b < 4; ++b)
                buf_store8(rout, lane * 4 + b < m ? (uint32_t)(pos - obase) + lane * 4 + b : kDrop, byte_of(x4, b));
            pos += m;
        } else {
            HC_PROF_BEGIN();
            pos += revert_block(x4, m, rc, dmask, rout, (uint32_t)(pos - obase), fgk.T.scratch, lane);
            HC_PROF_END(4);
        }
    }

    // blocks from i0 on; a block left unfinished at i (i0 <= i < its end) is finished first
    template <bool kWin>
    __device__ __forceinline__ void run(const Batch &bt, Idx i0, Idx i)
    {
        for (; i0 < n; i0 += 256, i = i0) {
            if (stopped()) break;
            block_start<kWin>(bt, i0);
            const Idx i1 = block_end(i0);
#if HC_DEC_BATCH
            // Batches pay where they take several symbols each; on flat alphabets (noise, -c
            // photos: codes at or past the tables' 8 bits) they stop short and the one-symbol
            // loop is faster (measured: C4 decode 2.02 s without batches, 3.52 s with them; a
            // lone wave waits out each batch's table reads). A block runs batches when the last
            // block that ran them took at least kBatchYield / 2 symbols per batch, and every 8th
            // block tries them again.
            if constexpr (kW <= 1) {
                if (btry) batch_on = 2 * bsym >= kBatchYield * btry;
                bsym = btry = 0;
                if (batch_on || ((uint32_t)(i0 >> 8) & 7u) == 0) {
                    decode<true>(i0, i, i1);
                    close_block(i0, i1);
                    continue;
                }
            }
            decode<false>(i0, i, i1);
#else
            decode(i0, i, i1);
#endif
            close_block(i0, i1);
        }
    }

    __device__ __forceinline__ void close(const Batch &bt)
    {
        if (consumed() > payload_bits) st = HC_ERR_HUFFMAN;  // ran past the payload
        if (fgk.bad) st = HC_ERR_DEVICE;
        if (st == 0 && pos > cap) st = HC_ERR_CAPACITY;
        if (lane == 0) {
            bt.status[sid] = (int32_t)st;
            bt.out_lens[sid] = (st == 0 || st == HC_ERR_CAPACITY) ? pos : 0;
        }
    }
};

template <int kW, int kDst, bool kSmall = false>
__global__ __launch_bounds__(64 * HC_WAVES) __attribute__((amdgpu_waves_per_eu(kWavesPerSimd<kW>))) void decode_kernel(Batch bt)
{
    __shared__ Tree<kW, true, false, kSmall> trees[kWaves];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t sid = blockIdx.x * kWaves + wv;
    if (sid >= bt.n) return;
    Dec<kW, kDst, kSmall> dec(trees[wv], lane);
    if (!dec.open(bt, sid)) return;
    // two copies of the block loop, as in the encoder: without window bookkeeping for streams
    // that fit one window (input and output), with it for the rest
    if (dec.one_window()) dec.template run<false>(bt, 0, 0);
    else dec.template run<true>(bt, 0, 0);
    dec.close(bt);
    trace_wave(sid, t0, lane);
    prof_store(sid, t0, dec.pacc + dec.fgk.pacc, lane);
}

}  // namespace

// streams that the table-mode encoder holds resident at once: 6 waves per SIMD (its LDS)
static uint32_t table_slots()
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return (uint32_t)cus * 24;
}

template <int kSrc>
static hipError_t launch_encode_src(const Batch &b, dim3 grid, dim3 block, hipStream_t st, hipStream_t aux)
{
    // every stream votes for its mode (enc_mode_kernel); the cache-mode launches run on the
    // caller's stream, each skipping the other mode's streams. The table-mode launches follow them
    // on the same stream, or -- when the caller gives a second stream -- run beside them there
    // (forked and joined by events), so that a mixed batch fills the GPU with both at once. The
    // library keeps no stream of its own.
    enc_mode_kernel<kSrc><<<(b.n + 3) / 4, 256, 0, st>>>(b, b.n <= table_slots() ? 1u : 0u, enc_tab());
    hipEvent_t fork = nullptr, join = nullptr;
    if (aux == st) aux = nullptr;
    if (aux && (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&join, hipEventDisableTiming) != hipSuccess))
        aux = nullptr;
    hipStream_t ts = st;  // the table-mode launches' stream
    if (aux && hipEventRecord(fork, st) == hipSuccess && hipStreamWaitEvent(aux, fork, 0) == hipSuccess) ts = aux;
    encode_kernel<0, kSrc><<<grid, block, 0, st>>>(b);
    encode_kernel<1, kSrc><<<grid, block, 0, st>>>(b);
    encode_kernel<2, kSrc><<<grid, block, 0, st>>>(b);
    encode_kernel<0, kSrc, true><<<grid, block, 0, ts>>>(b);
    encode_kernel<1, kSrc, true><<<grid, block, 0, ts>>>(b);
    hipError_t e = hipGetLastError();
    if (ts != st) {
        const hipError_t e1 = hipEventRecord(join, ts);
        const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(st, join, 0) : e1;
        if (e2 != hipSuccess) {
            // no join: wait for the side stream here, so that an error return never leaves
            // library work running unordered against the caller's buffers
            (void)hipStreamSynchronize(ts);
            if (e == hipSuccess) e = e2;
        }
    }
    // the small-alphabet streams last, after the join: its batch (grad: 8192 streams, one round of
    // waves) must not share the CUs with the other launches' workgroups while they start and exit
    // (launched first, beside the table launches: grad encode 1.23 -> 2.52 ms; after the cache
    // launches but before the join: 1.6 ms)
    encode_kernel<0, kSrc, false, true><<<grid, block, 0, st>>>(b);
    if (e == hipSuccess) e = hipGetLastError();
    if (fork) (void)hipEventDestroy(fork);  // (released once the recorded work completes)
    if (join) (void)hipEventDestroy(join);
    return e;
}

hipError_t launch_encode(const Batch &b0, EncSrc src, hipStream_t st, hipStream_t aux)
{
    if (b0.n == 0) return hipSuccess;
    Batch b = b0;
    b.min_tree = min_tree();
    const dim3 grid((b.n + kWaves - 1) / kWaves), block(64 * kWaves);
    // enc_mode_kernel marks each stream for the cache or the table launch; then one launch per
    // tree layout and mode, each stream coded by exactly one of them (tree_kind, the mark)
    switch (src) {
    case SRC_RAW: return launch_encode_src<SRC_RAW>(b, grid, block, st, aux);
    case SRC_RAW_DIFF: return launch_encode_src<SRC_RAW_DIFF>(b, grid, block, st, aux);
    default: return launch_encode_src<SRC_SYMBOLS>(b, grid, block, st, aux);
    }
}

hipError_t launch_decode(const Batch &b0, DecDst dst, hipStream_t st)
{
    if (b0.n == 0) return hipSuccess;
    Batch b = b0;
    b.min_tree = min_tree();
    b.dec_small = dec_small();
    const dim3 grid((b.n + kWaves - 1) / kWaves), block(64 * kWaves);
    // one launch per tree layout, then the small-alphabet streams' (dec_small_stream), each
    // stream decoded by exactly one of them
    if (dst == DST_RAW) {
        decode_kernel<0, DST_RAW><<<grid, block, 0, st>>>(b);
        decode_kernel<1, DST_RAW><<<grid, block, 0, st>>>(b);
        decode_kernel<2, DST_RAW><<<grid, block, 0, st>>>(b);
        decode_kernel<0, DST_RAW, true><<<grid, block, 0, st>>>(b);
    } else {
        decode_kernel<0, DST_SYMBOLS><<<grid, block, 0, st>>>(b);
        decode_kernel<1, DST_SYMBOLS><<<grid, block, 0, st>>>(b);
        decode_kernel<2, DST_SYMBOLS><<<grid, block, 0, st>>>(b);
        decode_kernel<0, DST_SYMBOLS, true><<<grid, block, 0, st>>>(b);
    }
    return hipGetLastError();
}

}  // namespace hc

#ifdef HC_DEBUG_HOOKS
extern "C" int hc_debug_set_window(uint32_t bytes)
{
    // a multiple of 256 in [4096, 2^30]: the descriptor windows of every later FGK launch
    uint32_t w = bytes < 4096u ? 4096u : (bytes > (1u << 30) ? (1u << 30) : bytes);
    w &= ~255u;
    return hipMemcpyToSymbol(HIP_SYMBOL(hc::g_window), &w, sizeof(w)) == hipSuccess ? 0 : HC_ERR_DEVICE;
}

extern "C" int hc_debug_set_min_tree(uint32_t kind)
{
    // 0 narrow, 1 wide, 2 huge: the smallest tree layout of every later FGK launch
    hc::g_min_tree = kind > 2 ? 2 : kind;
    return 0;
}

extern "C" int hc_debug_set_dec_small(uint32_t mode)
{
    // 0: by payload rate, 1: the small-alphabet decoder for every narrow stream, 2: for none
    hc::g_dec_small = mode > 2 ? 0 : mode;
    return 0;
}

extern "C" int hc_debug_set_enc_tab(uint32_t mode)
{
    // 0: per stream (sampled alphabet), 1: path cache for every stream, 2: tables for every
    // stream, 3: the small-alphabet kernel for every stream (narrow layout)
    hc::g_enc_tab = mode > 3 ? 0 : mode;
    return 0;
}

extern "C" int hc_debug_enc_votes(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens, uint32_t n,
                                  uint32_t flags, uint32_t low_occ, int32_t *status, void *stream)
{
    // enc_mode_kernel alone: status[i] = the vote (kModeCache -0x7A1 / kModeTables -0x7A0)
    hc::Batch b{};
    b.in = in;
    b.in_offs = in_offs;
    b.in_lens = in_lens;
    b.n = n;
    b.status = status;
    b.flags = flags;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) return 0;
    if (flags & HC_FLAG_DIFF) hc::enc_mode_kernel<hc::SRC_RAW_DIFF><<<(n + 3) / 4, 256, 0, st>>>(b, low_occ, 0u);
    else hc::enc_mode_kernel<hc::SRC_RAW><<<(n + 3) / 4, 256, 0, st>>>(b, low_occ, 0u);
    return hipGetLastError() == hipSuccess ? 0 : HC_ERR_DEVICE;
}

extern "C" int hc_debug_set_trace(void *dev_buf)
{
    uint64_t *p = static_cast<uint64_t *>(dev_buf);
    return hipMemcpyToSymbol(HIP_SYMBOL(hc::g_trace), &p, sizeof(p)) == hipSuccess ? 0 : HC_ERR_DEVICE;
}
#endif  // HC_DEBUG_HOOKS
