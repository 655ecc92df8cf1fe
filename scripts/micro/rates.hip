// rates.hip — throughput of single VALU instruction kinds at the FGK kernels' occupancy (8 waves
// per SIMD), relative to v_add_u32: 64 independent instructions per iteration (8 chains).
//   hipcc --offload-arch=gfx950 -O2 scripts/micro/rates.hip -o /tmp/rates && /tmp/rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
template <int T>
__global__ __launch_bounds__(256) void rates(uint32_t *out, int iters)
{
    uint32_t v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
    uint64_t w0 = v0, w1 = v1, w2 = v2, w3 = v3;
    uint32_t s = blockIdx.x & 7;
    uint64_t w0s = 0x5555555555555555ull ^ blockIdx.x;
    asm volatile("" : "+s"(s), "+s"(w0s));
    for (int it = 0; it < iters; ++it) {
        if (T == 0)
            asm volatile(R8("v_add_u32 %0, 1, %0\nv_add_u32 %1, 1, %1\nv_add_u32 %2, 1, %2\nv_add_u32 %3, 1, %3\n"
                            "v_add_u32 %0, 1, %0\nv_add_u32 %1, 1, %1\nv_add_u32 %2, 1, %2\nv_add_u32 %3, 1, %3\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        if (T == 1)
            asm volatile(R8("v_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\nv_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %4, %3\n"
                            "v_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\nv_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %4, %3\n")
                         : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3) : "s"(s));
        if (T == 2)
            asm volatile(R8("v_mul_lo_u32 %0, %0, %4\nv_mul_lo_u32 %1, %1, %4\nv_mul_lo_u32 %2, %2, %4\nv_mul_lo_u32 %3, %3, %4\n"
                            "v_mul_lo_u32 %0, %0, %4\nv_mul_lo_u32 %1, %1, %4\nv_mul_lo_u32 %2, %2, %4\nv_mul_lo_u32 %3, %3, %4\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
        if (T == 3)
            asm volatile(R8("v_mul_u32_u24 %0, %4, %0\nv_mul_u32_u24 %1, %4, %1\nv_mul_u32_u24 %2, %4, %2\nv_mul_u32_u24 %3, %4, %3\n"
                            "v_mul_u32_u24 %0, %4, %0\nv_mul_u32_u24 %1, %4, %1\nv_mul_u32_u24 %2, %4, %2\nv_mul_u32_u24 %3, %4, %3\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
        if (T == 4)
            asm volatile(R8("v_writelane_b32 %0, %4, 1\nv_writelane_b32 %1, %4, 2\nv_writelane_b32 %2, %4, 3\nv_writelane_b32 %3, %4, 4\n"
                            "v_writelane_b32 %0, %4, 5\nv_writelane_b32 %1, %4, 6\nv_writelane_b32 %2, %4, 7\nv_writelane_b32 %3, %4, 8\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
        if (T == 5)
            asm volatile(R8("v_bcnt_u32_b32 %0, %0, 0\nv_bcnt_u32_b32 %1, %1, 0\nv_bcnt_u32_b32 %2, %2, 0\nv_bcnt_u32_b32 %3, %3, 0\n"
                            "v_bcnt_u32_b32 %0, %0, 1\nv_bcnt_u32_b32 %1, %1, 1\nv_bcnt_u32_b32 %2, %2, 1\nv_bcnt_u32_b32 %3, %3, 1\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        if (T == 6)
            asm volatile(R8("v_and_b32 %0, 0x7f, %0\nv_and_b32 %1, 0x7f, %1\nv_and_b32 %2, 0x7f, %2\nv_and_b32 %3, 0x7f, %3\n"
                            "v_or_b32 %0, %4, %0\nv_or_b32 %1, %4, %1\nv_or_b32 %2, %4, %2\nv_or_b32 %3, %4, %3\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
        if (T == 7)
            asm volatile(R8("v_lshl_add_u32 %0, %0, 1, %4\nv_lshl_add_u32 %1, %1, 1, %4\nv_lshl_add_u32 %2, %2, 1, %4\nv_lshl_add_u32 %3, %3, 1, %4\n"
                            "v_lshl_add_u32 %0, %0, 2, %4\nv_lshl_add_u32 %1, %1, 2, %4\nv_lshl_add_u32 %2, %2, 2, %4\nv_lshl_add_u32 %3, %3, 2, %4\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
        if (T == 8)
            asm volatile(R8("v_cndmask_b32_e64 %0, %0, %1, %4\nv_cndmask_b32_e64 %1, %1, %2, %4\nv_cndmask_b32_e64 %2, %2, %3, %4\nv_cndmask_b32_e64 %3, %3, %0, %4\n"
                            "v_cndmask_b32_e64 %0, %0, %1, %4\nv_cndmask_b32_e64 %1, %1, %2, %4\nv_cndmask_b32_e64 %2, %2, %3, %4\nv_cndmask_b32_e64 %3, %3, %0, %4\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(w0s));
        if (T == 9)
            asm volatile(R8("v_cmp_lt_u32 vcc, %0, %1\nv_cmp_lt_u32 vcc, %1, %2\nv_cmp_lt_u32 vcc, %2, %3\nv_cmp_lt_u32 vcc, %3, %0\n"
                            "v_cmp_lt_u32 vcc, %0, %2\nv_cmp_lt_u32 vcc, %1, %3\nv_cmp_lt_u32 vcc, %2, %0\nv_cmp_lt_u32 vcc, %3, %1\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) :: "vcc");
        if (T == 10)
            asm volatile(R8("v_mov_b32_dpp %0, %1 row_shr:1\nv_mov_b32_dpp %1, %2 row_shr:1\nv_mov_b32_dpp %2, %3 row_shr:1\nv_mov_b32_dpp %3, %0 row_shr:1\n"
                            "v_mov_b32_dpp %0, %2 row_shr:1\nv_mov_b32_dpp %1, %3 row_shr:1\nv_mov_b32_dpp %2, %0 row_shr:1\nv_mov_b32_dpp %3, %1 row_shr:1\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        if (T == 11)
            asm volatile(R8("v_readfirstlane_b32 s8, %0\nv_readfirstlane_b32 s9, %1\nv_readfirstlane_b32 s10, %2\nv_readfirstlane_b32 s11, %3\n"
                            "v_readfirstlane_b32 s8, %1\nv_readfirstlane_b32 s9, %2\nv_readfirstlane_b32 s10, %3\nv_readfirstlane_b32 s11, %0\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) :: "s8", "s9", "s10", "s11");
        if (T == 12)
            asm volatile(R8("v_add_u32 %0, %4, %0\nv_add_u32 %1, %4, %1\nv_add_u32 %2, %4, %2\nv_add_u32 %3, %4, %3\n"
                            "v_sub_u32 %0, %0, %1\nv_sub_u32 %1, %1, %2\nv_sub_u32 %2, %2, %3\nv_sub_u32 %3, %3, %0\n")
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));
    }
    out[blockIdx.x * 256 + threadIdx.x] = v0 + v1 + v2 + v3 + (uint32_t)(w0 + w1 + w2 + w3);
}

int main()
{
    const int blocks = 2048, iters = 20000;  // 8 workgroups of 4 waves per CU on 256 CUs
    uint32_t *out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[13] = {"v_add_u32 (const)", "v_lshlrev_b64", "v_mul_lo_u32", "v_mul_u32_u24", "v_writelane_b32", "v_bcnt_u32_b32",
                             "v_and/or_b32", "v_lshl_add_u32", "v_cndmask_e64", "v_cmp_lt_u32", "v_mov_b32_dpp", "v_readfirstlane", "v_add/sub (vgpr)"};
    float base = 0;
    for (int t = 0; t < 13; ++t) {
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            switch (t) {
            case 0: rates<0><<<blocks, 256>>>(out, iters); break;
            case 1: rates<1><<<blocks, 256>>>(out, iters); break;
            case 2: rates<2><<<blocks, 256>>>(out, iters); break;
            case 3: rates<3><<<blocks, 256>>>(out, iters); break;
            case 4: rates<4><<<blocks, 256>>>(out, iters); break;
            case 5: rates<5><<<blocks, 256>>>(out, iters); break;
            case 6: rates<6><<<blocks, 256>>>(out, iters); break;
            case 7: rates<7><<<blocks, 256>>>(out, iters); break;
            case 8: rates<8><<<blocks, 256>>>(out, iters); break;
            case 9: rates<9><<<blocks, 256>>>(out, iters); break;
            case 10: rates<10><<<blocks, 256>>>(out, iters); break;
            case 11: rates<11><<<blocks, 256>>>(out, iters); break;
            case 12: rates<12><<<blocks, 256>>>(out, iters); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        if (t == 0) base = ms;
        const double inst = (double)blocks * 4 * iters * 64;  // wave instructions
        printf("%-16s %8.3f ms  %.2f x v_add  %.3f wave-instructions per cycle per CU\n", names[t], ms, ms / base,
               inst / 256 / (ms * 1e-3 * 2.4e9));
    }
    return 0;
}
