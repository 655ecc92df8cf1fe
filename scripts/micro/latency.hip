// latency.hip — dependent-chain latencies on gfx950 for the FGK kernels' design choices.
// (inline asm with SALU arithmetic declares "scc": an undeclared SCC write breaks the compiler's
// loop branch.) Each test runs a chain of 64 dependent steps (unrolled in asm) and reports cycles per step
// (s_memtime), for 1 wave on the chip and for 8 waves per SIMD on every CU (the kernels' shape).
//   hipcc --offload-arch=gfx950 -O2 scripts/micro/latency.hip -o /tmp/latency && /tmp/latency
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <vector>

#define STEPS 64
#define REPT ".rept 64\n"

template <int T, int LDSW = 4096, int NT = 256>
__global__ __launch_bounds__(NT) void chain(uint64_t *out, int iters, uint64_t *trace)
{
    __shared__ uint32_t lds[LDSW];
    for (int i = threadIdx.x; i < LDSW; i += blockDim.x) lds[i] = (i * 4) % (LDSW * 4);  // self-pointing words
    __syncthreads();
    uint32_t v = (threadIdx.x & 63) * 4 + (threadIdx.x >> 6) * 1024;  // per-wave row
    uint32_t s = 0, b1 = 1, b2 = 2, b3 = 3, a1 = 1, a2 = 2, a3 = 3, a4 = 4;
    uint64_t m = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (T == 0)  // VALU -> VALU
            asm volatile(REPT "v_add_u32 %0, 0, %0\n.endr" : "+v"(v));
        if (T == 1)  // SALU -> SALU
            asm volatile(REPT "s_add_u32 %0, %0, 0\n.endr" : "+s"(s) : : "scc");
        if (T == 2)  // LDS read -> address of the next (same row)
            asm volatile(REPT "ds_read_b32 %0, %0\ns_waitcnt lgkmcnt(0)\n.endr" : "+v"(v));
        if (T == 3)  // VALU -> SGPR -> SALU -> VALU
            asm volatile(REPT "v_readfirstlane_b32 %1, %0\ns_add_u32 %1, %1, 0\nv_mov_b32 %0, %1\n.endr"
                         : "+v"(v), "+s"(s) : : "scc");
        if (T == 4)  // VALU -> SGPR -> VALU (no SALU)
            asm volatile(REPT "v_readfirstlane_b32 %1, %0\nv_add_u32 %0, %1, 0\n.endr" : "+v"(v), "+s"(s));
        if (T == 5)  // v_cmp -> s_ff1 -> v_cmp -> v_cndmask  (the update's store mask)
            asm volatile(REPT "v_cmp_le_u32 %2, %0, 64\ns_ff1_i32_b64 %1, %2\nv_cmp_gt_u32 vcc, %1, %0\nv_cndmask_b32 %0, %0, %0, vcc\n.endr"
                         : "+v"(v), "+s"(s), "+s"(m) : : "vcc", "scc");
        if (T == 6)  // LDS read -> readfirstlane -> SALU -> v_mov -> LDS read
            asm volatile(REPT "ds_read_b32 %0, %0\ns_waitcnt lgkmcnt(0)\nv_readfirstlane_b32 %1, %0\ns_add_u32 %1, %1, 0\nv_mov_b32 %0, %1\n.endr"
                         : "+v"(v), "+s"(s) : : "scc");
        if (T == 7)  // LDS read -> VALU add -> LDS read (the VALU chase)
            asm volatile(REPT "ds_read_b32 %0, %0\ns_waitcnt lgkmcnt(0)\nv_add_u32 %0, 0, %0\n.endr" : "+v"(v));
        if (T == 8)  // (unused)
            asm volatile("" : "+v"(v));
        if (T == 10)  // throughput: 4 independent VALU per step
            asm volatile(REPT "v_add_u32 %0, 0, %0\nv_add_u32 %1, 0, %1\nv_add_u32 %2, 0, %2\nv_add_u32 %3, 0, %3\n.endr"
                         : "+v"(v), "+v"(a1), "+v"(a2), "+v"(a3));
        if (T == 11)  // throughput: 4 independent SALU per step
            asm volatile(REPT "s_add_u32 %0, %0, 0\ns_add_u32 %1, %1, 0\ns_add_u32 %2, %2, 0\ns_add_u32 %3, %3, 0\n.endr"
                         : "+s"(s), "+s"(b1), "+s"(b2), "+s"(b3) : : "scc");
        if (T == 12)  // throughput: 2 VALU + 2 SALU independent per step
            asm volatile(REPT "v_add_u32 %0, 0, %0\ns_add_u32 %2, %2, 0\nv_add_u32 %1, 0, %1\ns_add_u32 %3, %3, 0\n.endr"
                         : "+v"(v), "+v"(a1), "+s"(s), "+s"(b1) : : "scc");
        if (T == 13)  // throughput: 4 independent LDS reads per step (distinct lanes, one wait)
            asm volatile(REPT "ds_read_b32 %1, %0\nds_read_b32 %2, %0 offset:256\nds_read_b32 %3, %0 offset:512\nds_read_b32 %4, %0 offset:768\ns_waitcnt lgkmcnt(0)\n.endr"
                         : "+v"(v), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4));
        if (T == 9)  // SALU -> VALU (s_add then v_add reading it)
            asm volatile(REPT "s_add_u32 %1, %1, 0\nv_add_u32 %0, %1, %0\n.endr" : "+v"(v), "+s"(s) : : "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (trace && (threadIdx.x & 63) == 0) {
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        hw = (hw & 0xFFFFu) | ((xcc & 0xFu) << 16);
        trace[3 * w] = t0;
        trace[3 * w + 1] = t1;
        trace[3 * w + 2] = hw;
    }
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] =
            (t1 - t0) + ((v + a1 + a2 + a3 + a4 + s + b1 + b2 + b3) & 1);
}

template <int T, int LDSW = 4096>
double run(int blocks, int iters)
{
    uint64_t *d;
    const int waves = blocks * 4;
    hipMalloc(&d, waves * sizeof(uint64_t));
    chain<T, LDSW><<<blocks, 256>>>(d, iters, nullptr);  // warm
    chain<T, LDSW><<<blocks, 256>>>(d, iters, nullptr);
    hipDeviceSynchronize();
    uint64_t *h = new uint64_t[waves];
    hipMemcpy(h, d, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < waves; ++i) sum += (double)h[i];
    delete[] h;
    hipFree(d);
    return sum / waves / ((double)iters * STEPS);
}

// residency: how many of a launch's waves ran at the same time on one SIMD (max over SIMDs)
template <int LDSW, int NT = 256>
void residency(int blocks, int iters)
{
    const int waves = blocks * (NT / 64);
    uint64_t *d, *tr;
    (void)hipMalloc(&d, waves * sizeof(uint64_t));
    (void)hipMalloc(&tr, 3 * waves * sizeof(uint64_t));
    chain<10, LDSW, NT><<<blocks, NT>>>(d, iters, tr);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h(3 * waves);
    (void)hipMemcpy(h.data(), tr, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
    // HW_ID: wave_id [3:0], simd_id [5:4], cu_id [11:8], sh_id [12], se_id [15:13] (gfx9)
    std::map<uint32_t, std::vector<std::pair<uint64_t, int>>> ev;
    uint64_t t_lo = ~0ull, t_hi = 0;
    for (int w = 0; w < waves; ++w) {
        const uint32_t hw = (uint32_t)h[3 * w + 2];
        const uint32_t key = hw & ~0xFu;  // xcc, se, sh, cu, simd: everything but the wave slot
        ev[key].push_back({h[3 * w], +1});
        ev[key].push_back({h[3 * w + 1], -1});
        if ((hw >> 16) == 0) {
            t_lo = std::min(t_lo, h[3 * w]);
            t_hi = std::max(t_hi, h[3 * w + 1]);
        }
    }
    int best = 0;
    double mean_peak = 0;
    for (auto &kv : ev) {
        auto v = kv.second;
        std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
        int cur = 0, peak = 0;
        for (auto &e : v) peak = std::max(peak, cur += e.second);
        best = std::max(best, peak);
        mean_peak += peak;
    }
    printf("%4d thr, LDS %6d B/WG: %d waves over %zu SIMD keys (XCD ids alias), max %d / mean %.2f concurrent waves per key, "
           "span (XCC 0) %.0f cycles\n", NT, LDSW * 4, waves, ev.size(), best, mean_peak / ev.size(), (double)(t_hi - t_lo));
    (void)hipFree(d);
    (void)hipFree(tr);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[] = {"VALU->VALU", "SALU->SALU", "LDS read chain", "VALU->SGPR->SALU->VALU",
                           "VALU->SGPR->VALU", "v_cmp->s_ff1->v_cmp->v_cndmask", "LDS->readfirstlane->SALU->VALU->LDS",
                           "LDS->VALU->LDS", "(unused)", "SALU->VALU", "thru: 4 indep VALU", "thru: 4 indep SALU",
                           "thru: 2 VALU + 2 SALU", "thru: 4 indep ds_read_b32"};
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    printf("%s: sharedMemPerBlock %zu, maxSharedMemoryPerMultiProcessor %zu, regsPerMultiprocessor %d, "
           "maxThreadsPerMultiProcessor %d, clock %d kHz\n", pr.gcnArchName, pr.sharedMemPerBlock,
           pr.maxSharedMemoryPerMultiProcessor, pr.regsPerMultiprocessor, pr.maxThreadsPerMultiProcessor, pr.clockRate);
    residency<64>(cus * 8, 2000);
    residency<256>(cus * 8, 2000);
    residency<512>(cus * 8, 2000);
    residency<1024>(cus * 8, 2000);
    residency<2048>(cus * 8, 2000);
    residency<1280, 64>(cus * 32, 2000);       // 1 wave, 5 KB
    residency<10240, 512>(cus * 4, 2000);      // 8 waves, 40 KB
    residency<20480, 1024>(cus * 2, 2000);     // 16 waves, 80 KB
    residency<10240, 1024>(cus * 2, 2000);     // 16 waves, 40 KB
    fflush(stdout);
    printf("cycles per dependent step (s_memtime units), %d CUs\n", cus);
    printf("%-40s %14s %18s\n", "chain", "1 WG (4 waves)", "8 WG/CU (32 w/CU)");
    fflush(stdout);
#define RUN(T)                                                                        \
    {                                                                                 \
        const double a = run<T>(1, 200), b = run<T>(cus * 8, 2000);                   \
        printf("%-40s %14.1f %18.1f\n", names[T], a, b);                              \
        fflush(stdout);                                                               \
    }
    if (getenv("LAT_CHAINS")) {
        RUN(0) RUN(1) RUN(2) RUN(9) RUN(7) RUN(4) RUN(3) RUN(6) RUN(5) RUN(10) RUN(11) RUN(12) RUN(13)
    }
    // issue throughput with full residency (no LDS: 8 waves per SIMD, checked above): per wave
    // cycles per step of 4 independent instructions -> instructions per cycle per SIMD / CU
    printf("throughput at 8 waves/SIMD (LDS-free kernels):\n");
#define THRU(T, what)                                                                                \
    {                                                                                                \
        const double c1 = run<T, 16>(1, 2000), c8 = run<T, 16>(cus * 8, 2000);                      \
        printf("  %-28s 1 wave/SIMD: %5.1f cyc/step; 8 waves/SIMD: %5.1f cyc/step = %.2f/cycle/SIMD, %.2f/cycle/CU\n", \
               what, c1, c8, 8 * 4 / c8, 32 * 4 / c8);                                               \
        fflush(stdout);                                                                              \
    }
    THRU(10, "4 indep VALU") THRU(11, "4 indep SALU") THRU(12, "2 VALU + 2 SALU")
    return 0;
}
