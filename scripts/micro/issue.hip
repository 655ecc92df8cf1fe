// issue.hip — instruction throughput per CU on gfx950 at the FGK kernels' occupancy (8 waves per
// SIMD, 32 per CU): independent VALU, SALU, and an even VALU/SALU mix, 64 instructions per
// iteration (VALU + ds_read_b32: 4 waits per iteration besides). Reports instructions per cycle
// per CU (2.4 GHz assumed from the kernel time).
//   hipcc --offload-arch=gfx950 -O2 scripts/micro/issue.hip -o /tmp/issue && /tmp/issue
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int T>
__global__ __launch_bounds__(256) void issue(uint32_t *out, int iters)
{
    uint32_t v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    __shared__ uint32_t lds[256 * 8];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint32_t la = (threadIdx.x & 63) * 4;
    uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    for (int it = 0; it < iters; ++it) {
        if (T == 0)
            asm volatile(".rept 8\nv_add_u32 %0, 1, %0\nv_add_u32 %1, 1, %1\nv_add_u32 %2, 1, %2\nv_add_u32 %3, 1, %3\n"
                         "v_add_u32 %4, 1, %4\nv_add_u32 %5, 1, %5\nv_add_u32 %6, 1, %6\nv_add_u32 %7, 1, %7\n.endr"
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
        if (T == 1)
            asm volatile(".rept 8\ns_add_u32 %0, 1, %0\ns_add_u32 %1, 1, %1\ns_add_u32 %2, 1, %2\ns_add_u32 %3, 1, %3\n"
                         "s_add_u32 %4, 1, %4\ns_add_u32 %5, 1, %5\ns_add_u32 %6, 1, %6\ns_add_u32 %7, 1, %7\n.endr"
                         : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
                         :
                         : "scc");
        if (T == 2)
            asm volatile(".rept 8\nv_add_u32 %0, 1, %0\ns_add_u32 %4, 1, %4\nv_add_u32 %1, 1, %1\ns_add_u32 %5, 1, %5\n"
                         "v_add_u32 %2, 1, %2\ns_add_u32 %6, 1, %6\nv_add_u32 %3, 1, %3\ns_add_u32 %7, 1, %7\n.endr"
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
                         :
                         : "scc");
        if (T == 3)  // VALU with LDS reads, 1:1 (waits once per 8 reads)
            asm volatile(".rept 4\nv_add_u32 %0, 1, %0\nds_read_b32 %4, %8\nv_add_u32 %1, 1, %1\nds_read_b32 %5, %8 offset:256\n"
                         "v_add_u32 %2, 1, %2\nds_read_b32 %6, %8 offset:512\nv_add_u32 %3, 1, %3\nds_read_b32 %7, %8 offset:768\n"
                         "v_add_u32 %0, 1, %0\nds_read_b32 %4, %8 offset:1024\nv_add_u32 %1, 1, %1\nds_read_b32 %5, %8 offset:1280\n"
                         "v_add_u32 %2, 1, %2\nds_read_b32 %6, %8 offset:1536\nv_add_u32 %3, 1, %3\nds_read_b32 %7, %8 offset:1792\n"
                         "s_waitcnt lgkmcnt(0)\n.endr"
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
                         : "v"(la));
    }
    v0 += l0 + l1 + l2 + l3;
    out[blockIdx.x * 256 + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
}

int main()
{
    const int blocks = 2048, iters = 20000;  // 8 workgroups of 4 waves per CU on 256 CUs
    uint32_t *out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[4] = {"VALU", "SALU", "VALU+SALU 1:1", "VALU+LDS 1:1"};
    for (int t = 0; t < 4; ++t) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (t == 0) issue<0><<<blocks, 256>>>(out, iters);
            if (t == 1) issue<1><<<blocks, 256>>>(out, iters);
            if (t == 2) issue<2><<<blocks, 256>>>(out, iters);
            if (t == 3) issue<3><<<blocks, 256>>>(out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double insts = (double)blocks * 4 * iters * 64 / 256;  // per CU
            if (rep) printf("%-14s %.3f ms  %.3f instructions / cycle / CU\n", names[t], ms, insts / (ms * 1e-3 * 2.4e9));
        }
    }
    return 0;
}
