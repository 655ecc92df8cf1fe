// hc_floor.hip — `hc-floor`: the per-process floor of ANY HIP program on a box, next to which
// bench.py's C1 line prices the drop-in CLI (bin/huffman-codec, one file per process like the
// reference's main.cpp:152-221). It does what every GPU process must before its first result:
// process start with the HIP runtime linked, HIP start-up (device enumeration, the context of
// device 0), one empty kernel launched and waited for (its code object loaded, a queue created),
// exit. Whatever the CLI costs above this per file is the codec's own.
//
// HC_CLI_TIMES=1: one stderr line "hc-times hip_init_ms=.. first_launch_ms=.." (the phases inside
// the process, in the CLI's format).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void floor_kernel(int *p)
{
    if (p && threadIdx.x == 0) *p = 1;  // never taken (p is null): an empty kernel the compiler keeps
}

static double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main()
{
    const char *env = std::getenv("HC_CLI_TIMES");
    const bool times = env && env[0] == '1';
    auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || hipSetDevice(0) != hipSuccess) {
        std::fprintf(stderr, "hc-floor: no HIP device\n");
        return 1;
    }
    const double t_init = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    floor_kernel<<<1, 64>>>(nullptr);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::fprintf(stderr, "hc-floor: launch failed\n");
        return 1;
    }
    const double t_launch = ms_since(t0);
    if (times) std::fprintf(stderr, "hc-times hip_init_ms=%.3f first_launch_ms=%.3f\n", t_init, t_launch);
    return 0;
}
