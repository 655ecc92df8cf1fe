// first_call.cpp — where the drop-in CLI's first call spends its one-time cost (diagnostic for
// bench.py configs.C1): HIP start-up, a first device allocation and copy, a first tiny coding
// call (code objects loaded at the first launch, the library's first buffers), then the file's
// coding twice. Build: bash scripts/micro/build_first_call.sh; run: scripts/micro/first_call FILE
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <vector>

#include "hcodec.h"

static double ms(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    std::ifstream f(argv[1], std::ios::binary);
    const std::vector<uint8_t> in((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const bool first_alloc = argc < 3 || argv[2][0] != 'n';
    auto t = std::chrono::steady_clock::now();
    const int ok = hc_device_ok();
    std::printf("device_ok %d %.1f ms\n", ok, ms(t));
    if (first_alloc) {
        t = std::chrono::steady_clock::now();
        void *p = nullptr;
        (void)hipMalloc(&p, 1 << 20);
        std::printf("hipMalloc 1 MiB %.1f ms\n", ms(t));
        t = std::chrono::steady_clock::now();
        (void)hipMemcpy(p, in.data(), 4096, hipMemcpyHostToDevice);
        std::printf("first H2D 4 KiB %.1f ms\n", ms(t));
        if (argv[2] && argv[2][0] == 'b') {  // then a file-sized copy each way
            t = std::chrono::steady_clock::now();
            (void)hipMemcpy(p, in.data(), in.size() < (1u << 20) ? in.size() : (1u << 20), hipMemcpyHostToDevice);
            std::printf("first H2D of the file %.1f ms\n", ms(t));
            std::vector<uint8_t> h(1 << 20);
            t = std::chrono::steady_clock::now();
            (void)hipMemcpy(h.data(), p, 1 << 17, hipMemcpyDeviceToHost);
            std::printf("first D2H 128 KiB %.1f ms\n", ms(t));
        }
        (void)hipFree(p);
    }
    std::vector<uint8_t> out(hc_compress_bound(in.size(), 0));
    uint64_t n = 0;
    t = std::chrono::steady_clock::now();
    (void)hc_compress(in.data(), 1, 1, 0, 512, out.data(), out.size(), &n);
    std::printf("tiny -c -m (1 byte) %.1f ms\n", ms(t));
    for (int k = 0; k < 3; ++k) {
        t = std::chrono::steady_clock::now();
        (void)hc_compress(in.data(), in.size(), 1, 0, 512, out.data(), out.size(), &n);
        std::printf("file -c -m #%d %.1f ms (%llu bytes)\n", k, ms(t), (unsigned long long)n);
    }
    std::vector<uint8_t> enc(out.begin(), out.begin() + (long)n);
    uint8_t *back = nullptr;
    uint64_t m = 0;
    t = std::chrono::steady_clock::now();
    (void)hc_decompress_alloc(enc.data(), 9, &back, &m);
    hc_free(back);
    std::printf("tiny -d (header only) %.1f ms\n", ms(t));
    for (int k = 0; k < 3; ++k) {
        t = std::chrono::steady_clock::now();
        (void)hc_decompress_alloc(enc.data(), enc.size(), &back, &m);
        std::printf("file -d #%d %.1f ms (%llu bytes)\n", k, ms(t), (unsigned long long)m);
        hc_free(back);
    }
    return 0;
}
