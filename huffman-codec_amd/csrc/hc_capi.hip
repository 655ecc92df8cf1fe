// hc_capi.hip — the C ABI of include/hcodec.h on top of the gfx950 kernels.
//
// The single-buffer entry points follow huffCompress / huffDecompress (main.cpp:39-128): same
// stages in the same order, same status numbers; the stages themselves run on the device.
// There is no host fallback: every stage is a HIP kernel, and without a device the calls fail
// with HC_ERR_DEVICE.
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <utility>
#include <vector>

#include "hc_internal.h"

namespace {

using hc::Batch;

// Device scratch of the single-buffer API. A call takes buffers from a per-device free list
// (hipMalloc only when none is large enough) and gives them back at its end, so a process that
// codes file after file (the CLI, C2) stops allocating after its first call. The list keeps at
// most kKeepBytes per device (larger leftovers are freed at once) and hc_release_cached() frees
// it. It caches memory only: no result depends on it, and concurrent calls never share a buffer.
constexpr uint64_t kKeepBytes = 1ull << 30;
struct FreeList {
    std::mutex mu;
    std::vector<std::pair<void *, uint64_t>> bufs[64];  // per device: (pointer, bytes)
    uint64_t kept[64] = {};
};
FreeList &free_list()
{
    static FreeList *const f = new FreeList;  // never destroyed: the HIP runtime may be gone at exit
    return *f;
}

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    int dev = -1;
    ~DevBuf() { give_back(); }
    void give_back()
    {
        if (!p) return;
        // the single-buffer API runs on the null stream; a call that returns early (an error
        // after an asynchronous launch) may still have kernels writing this buffer, so wait for
        // them before the next call can take it
        (void)hipStreamSynchronize(nullptr);
        FreeList &f = free_list();
        {
            std::lock_guard<std::mutex> lk(f.mu);
            if (dev >= 0 && dev < 64 && f.kept[dev] + cap <= kKeepBytes) {
                f.bufs[dev].emplace_back(p, cap);
                f.kept[dev] += cap;
                p = nullptr;
            }
        }
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    // at least n bytes: the smallest cached buffer that fits, else a new one (one retry after
    // freeing the cache when the device is short of memory)
    hipError_t alloc(uint64_t n)
    {
        give_back();
        n = n < 16 ? 16 : (n + 255) & ~255ull;
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
        if (dev >= 0 && dev < 64) {
            FreeList &f = free_list();
            std::lock_guard<std::mutex> lk(f.mu);
            auto &v = f.bufs[dev];
            size_t best = v.size();
            for (size_t k = 0; k < v.size(); ++k)
                if (v[k].second >= n && (best == v.size() || v[k].second < v[best].second)) best = k;
            if (best != v.size()) {
                p = v[best].first;
                cap = v[best].second;
                f.kept[dev] -= cap;
                v.erase(v.begin() + (long)best);
                return hipSuccess;
            }
        }
        hipError_t e = hipMalloc(&p, n);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            hc_release_cached();
            e = hipMalloc(&p, n);
        }
        cap = e == hipSuccess ? n : 0;
        if (e != hipSuccess) p = nullptr;
        return e;
    }
    template <class T>
    T *as() const
    {
        return reinterpret_cast<T *>(p);
    }
};

#define HC_CK(x)                                 \
    do {                                         \
        if ((x) != hipSuccess) return HC_ERR_DEVICE; \
    } while (0)

bool aligned4(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

// worst-case FGK symbols produced from n input bytes
uint64_t max_symbols(uint64_t n, int use_adapt)
{
    if (!use_adapt) return n + n / 3 + 2;
    // adaptive stream: header 24 + one bit per block, MNP-5 of a block of L bytes <= 4L/3 + 1,
    // blocks <= n / 16 (W, H >= 8)
    return n + n / 3 + n / 16 + n / 128 + 64;
}

// One stream through a batch launch of size 1. Per-stream scalars live in a small device
// block: [in_off, in_len, out_off, out_cap, out_len, status].
int run_single(bool encode, int mode, const uint8_t *d_in, uint64_t in_len, uint8_t *d_out,
               uint64_t out_cap, uint32_t flags, uint64_t *out_len, int *status, hipStream_t st)
{
    DevBuf meta;
    HC_CK(meta.alloc(8 * sizeof(uint64_t)));
    uint64_t h[8] = {0, in_len, 0, out_cap, 0, 0, 0, 0};
    HC_CK(hipMemcpyAsync(meta.p, h, sizeof(h), hipMemcpyHostToDevice, st));
    uint64_t *m = meta.as<uint64_t>();
    Batch b;
    b.in = d_in;
    b.in_offs = m + 0;
    b.in_lens = m + 1;
    b.n = 1;
    b.out = d_out;
    b.out_offs = m + 2;
    b.out_caps = m + 3;
    b.out_lens = m + 4;
    b.status = reinterpret_cast<int32_t *>(m + 5);
    b.flags = flags;
    hipError_t e = encode ? hc::launch_encode(b, (hc::EncSrc)mode, st)
                          : hc::launch_decode(b, (hc::DecDst)mode, st);
    HC_CK(e);
    HC_CK(hipMemcpyAsync(h, meta.p, sizeof(h), hipMemcpyDeviceToHost, st));
    HC_CK(hipStreamSynchronize(st));
    *out_len = h[4];
    *status = (int32_t)h[5];
    return HC_OK;
}

// One matrix / stream through the batched adaptive kernels (a batch of 1 with its workspace).
int run_adapt_single(bool encode, const uint8_t *d_in, uint64_t in_len, uint64_t width, uint32_t flags,
                     uint8_t *d_out, uint64_t out_cap, uint64_t *out_len, int *status, hipStream_t st)
{
    DevBuf meta, work;
    HC_CK(meta.alloc(8 * sizeof(uint64_t)));
    uint64_t h[8] = {0, in_len, width, 0, out_cap, 0, 0, 0};
    HC_CK(hipMemcpyAsync(meta.p, h, sizeof(h), hipMemcpyHostToDevice, st));
    uint64_t *m = meta.as<uint64_t>();
    Batch b;
    b.in = d_in;
    b.in_offs = m + 0;
    b.in_lens = m + 1;
    b.n = 1;
    b.out = d_out;
    b.out_offs = m + 3;
    b.out_caps = m + 4;
    b.out_lens = m + 5;
    b.status = reinterpret_cast<int32_t *>(m + 6);
    b.flags = flags;
    const uint64_t wb = encode ? hc::adapt_encode_work_bound(in_len, 1) : hc::adapt_decode_work_bound(in_len, out_cap, 1);
    HC_CK(work.alloc(wb));
    HC_CK(encode ? hc::adapt_encode_batch(b, m + 2, work.p, wb, st) : hc::adapt_decode_batch(b, work.p, wb, st));
    HC_CK(hipMemcpyAsync(h, meta.p, sizeof(h), hipMemcpyDeviceToHost, st));
    HC_CK(hipStreamSynchronize(st));
    *out_len = h[5];
    *status = (int32_t)h[6];
    return HC_OK;
}

int compress_impl(const uint8_t *in, uint64_t n, int use_diff, int use_adapt, uint64_t width,
                  std::vector<uint8_t> &res)
{
    if (width == 0) return HC_ERR_WIDTH;                  // main.cpp:195-199
    if (use_adapt && n % width != 0) return HC_ERR_MATRIX_SIZE;  // main.cpp:54-58
    const uint64_t height = n / width;
    if (use_adapt && (width < 8 || height < 8)) return HC_ERR_DIMS;  // transform.cpp:300-304
    if (!hc_device_ok()) return HC_ERR_DEVICE;
    hipStream_t st = nullptr;
    DevBuf din, dout;
    HC_CK(din.alloc(n + 16));
    if (n) HC_CK(hipMemcpyAsync(din.p, in, n, hipMemcpyHostToDevice, st));
    uint64_t len = 0;
    int status = 0;
    const uint64_t cap = hc_compress_bound(n, use_adapt);
    HC_CK(dout.alloc(cap));
    if (!use_adapt) {
        const int rc = run_single(true, use_diff ? hc::SRC_RAW_DIFF : hc::SRC_RAW, din.as<uint8_t>(), n,
                                  dout.as<uint8_t>(), cap, 0, &len, &status, st);
        if (rc) return rc;
    } else {
        // main.cpp:62-71: [diff] -> adaptive block RLE -> FGK, through the batched kernels
        const int rc = run_adapt_single(true, din.as<uint8_t>(), n, width, use_diff ? HC_FLAG_DIFF : 0u,
                                        dout.as<uint8_t>(), cap, &len, &status, st);
        if (rc) return rc;
    }
    if (status) return status;
    res.resize(len);
    if (len) HC_CK(hipMemcpy(res.data(), dout.p, len, hipMemcpyDeviceToHost));
    return HC_OK;
}

int decompress_impl(const uint8_t *in, uint64_t n, std::vector<uint8_t> &res)
{
    if (n < 9) return HC_ERR_HEADER;  // main.cpp:99-104
    if (!hc_device_ok()) return HC_ERR_DEVICE;
    uint64_t count = 0;
    for (int i = 7; i >= 0; --i) count = (count << 8) | in[i];
    const uint32_t flags = in[8];
    const uint64_t avail = (n - 9) * 8;
    if (count > (avail >= 8 ? avail - 7 : 0)) return HC_ERR_HUFFMAN;
    hipStream_t st = nullptr;
    DevBuf din;
    HC_CK(din.alloc(n + 16));
    HC_CK(hipMemcpyAsync(din.p, in, n, hipMemcpyHostToDevice, st));
    uint64_t len = 0;
    int status = 0;
    if (!(flags & HC_FLAG_ADAPT)) {
        // fused FGK -> RLE revert -> [diff revert]; the raw size is unknown up front, so guess,
        // and rerun with the exact size the device reports if the guess was short
        const uint64_t most = count * 65 + 8;  // any 4 symbols expand to <= 258 bytes
        uint64_t cap = n * 16 > (1u << 20) ? n * 16 : (1u << 20);
        if (cap > most) cap = most;
        for (int pass = 0; pass < 2; ++pass) {
            DevBuf dout;
            HC_CK(dout.alloc(cap));
            const int rc = run_single(false, hc::DST_RAW, din.as<uint8_t>(), n, dout.as<uint8_t>(), cap, 0,
                                      &len, &status, st);
            if (rc) return rc;
            if (status == HC_ERR_CAPACITY && pass == 0) {
                cap = len;
                continue;
            }
            if (status) return status;
            res.resize(len);
            if (len) HC_CK(hipMemcpy(res.data(), dout.p, len, hipMemcpyDeviceToHost));
            return HC_OK;
        }
        return HC_ERR_CAPACITY;
    }
    // main.cpp:114-125: FGK -> adaptive block revert -> [diff revert]; the matrix size is in
    // the adaptive header, so guess, and rerun with the size the device reports if short
    // W H <= 64.5 count for adaptive streams too (4 symbols expand to <= 258 bytes)
    const uint64_t most = count * 65 + 8;
    uint64_t cap = n * 16 > (1u << 20) ? n * 16 : (1u << 20);
    if (cap > most) cap = most;
    for (int pass = 0; pass < 2; ++pass) {
        DevBuf dout;
        HC_CK(dout.alloc(cap));
        const int rc = run_adapt_single(false, din.as<uint8_t>(), n, 0, 0, dout.as<uint8_t>(), cap, &len, &status, st);
        if (rc) return rc;
        if (status == HC_ERR_CAPACITY && pass == 0) {
            cap = len;
            continue;
        }
        if (status) return status;
        res.resize(len);
        if (len) HC_CK(hipMemcpy(res.data(), dout.p, len, hipMemcpyDeviceToHost));
        return HC_OK;
    }
    return HC_ERR_CAPACITY;
}

}  // namespace

extern "C" {

uint64_t hc_compress_bound(uint64_t in_len, int use_adapt)
{
    // <= 41 bits per FGK symbol below 2^22 symbols (depth <= 32 + NYT + 8 raw bits, sibling
    // property => Huffman depth bound); 48 bits leaves margin, plus header and word slack
    return 16 + max_symbols(in_len, use_adapt) * 6;
}

int hc_compress(const uint8_t *in, uint64_t in_len, int use_diff, int use_adapt, uint64_t width,
                uint8_t *out, uint64_t out_cap, uint64_t *out_len)
{
    if ((!in && in_len) || !out_len) return HC_ERR_ARG;
    std::vector<uint8_t> res;
    const int rc = compress_impl(in, in_len, use_diff, use_adapt, width, res);
    if (rc) return rc;
    *out_len = res.size();
    if (res.size() > out_cap) return HC_ERR_CAPACITY;
    if (!res.empty()) memcpy(out, res.data(), res.size());
    return HC_OK;
}

int hc_decompress(const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t out_cap,
                  uint64_t *out_len)
{
    if ((!in && in_len) || !out_len) return HC_ERR_ARG;
    std::vector<uint8_t> res;
    const int rc = decompress_impl(in, in_len, res);
    if (rc) return rc;
    *out_len = res.size();
    if (res.size() > out_cap) return HC_ERR_CAPACITY;
    if (!res.empty()) memcpy(out, res.data(), res.size());
    return HC_OK;
}

int hc_decompress_alloc(const uint8_t *in, uint64_t in_len, uint8_t **out, uint64_t *out_len)
{
    if ((!in && in_len) || !out || !out_len) return HC_ERR_ARG;
    *out = nullptr;
    std::vector<uint8_t> res;
    const int rc = decompress_impl(in, in_len, res);
    if (rc) return rc;
    *out = static_cast<uint8_t *>(malloc(res.size() ? res.size() : 1));
    if (!res.empty()) memcpy(*out, res.data(), res.size());
    *out_len = res.size();
    return HC_OK;
}

void hc_free(void *p) { free(p); }

int hc_compress_batch(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens,
                      uint32_t n_streams, uint32_t flags, uint8_t *out, const uint64_t *out_offs,
                      const uint64_t *out_caps, uint64_t *out_lens, int32_t *status, void *stream)
{
    return hc_compress_batch_aux(in, in_offs, in_lens, n_streams, flags, out, out_offs, out_caps, out_lens, status,
                                 stream, nullptr);
}

int hc_compress_batch_aux(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens,
                          uint32_t n_streams, uint32_t flags, uint8_t *out, const uint64_t *out_offs,
                          const uint64_t *out_caps, uint64_t *out_lens, int32_t *status, void *stream,
                          void *aux_stream)
{
    if (n_streams == 0) return HC_OK;
    if (!in || !in_offs || !in_lens || !out || !out_offs || !out_caps || !out_lens || !status)
        return HC_ERR_ARG;
    if (flags & ~HC_FLAG_DIFF) return HC_ERR_ARG;
    if (!aligned4(in) || !aligned4(out)) return HC_ERR_ARG;
    Batch b{in, in_offs, in_lens, n_streams, out, out_offs, out_caps, out_lens, status, flags};
    const hipError_t e = hc::launch_encode(b, (flags & HC_FLAG_DIFF) ? hc::SRC_RAW_DIFF : hc::SRC_RAW,
                                           static_cast<hipStream_t>(stream), static_cast<hipStream_t>(aux_stream));
    return e == hipSuccess ? HC_OK : HC_ERR_DEVICE;
}

int hc_decompress_batch(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens,
                        uint32_t n_streams, uint8_t *out, const uint64_t *out_offs,
                        const uint64_t *out_caps, uint64_t *out_lens, int32_t *status,
                        void *stream)
{
    if (n_streams == 0) return HC_OK;
    if (!in || !in_offs || !in_lens || !out || !out_offs || !out_caps || !out_lens || !status)
        return HC_ERR_ARG;
    if (!aligned4(in) || !aligned4(out)) return HC_ERR_ARG;
    Batch b{in, in_offs, in_lens, n_streams, out, out_offs, out_caps, out_lens, status, 0};
    const hipError_t e = hc::launch_decode(b, hc::DST_RAW, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? HC_OK : HC_ERR_DEVICE;
}

uint64_t hc_adapt_compress_work_bound(uint64_t total_in_bytes, uint32_t n_streams)
{
    return hc::adapt_encode_work_bound(total_in_bytes, n_streams);
}

uint64_t hc_adapt_decompress_work_bound(uint64_t total_in_bytes, uint64_t total_out_bytes, uint32_t n_streams)
{
    return hc::adapt_decode_work_bound(total_in_bytes, total_out_bytes, n_streams);
}

int hc_compress_adapt_batch(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens,
                            const uint64_t *widths, uint32_t n_streams, uint32_t flags, uint8_t *out,
                            const uint64_t *out_offs, const uint64_t *out_caps, uint64_t *out_lens,
                            int32_t *status, void *work, uint64_t work_bytes, void *stream)
{
    if (n_streams == 0) return HC_OK;
    if (!in || !in_offs || !in_lens || !widths || !out || !out_offs || !out_caps || !out_lens || !status || !work)
        return HC_ERR_ARG;
    if (flags & ~(HC_FLAG_DIFF | HC_FLAG_ADAPT)) return HC_ERR_ARG;
    if (!aligned4(in) || !aligned4(out) || (reinterpret_cast<uintptr_t>(work) & 15u)) return HC_ERR_ARG;
    // the workspace's fixed part (per-stream metadata, work lists) must fit whatever the sizes
    if (work_bytes < hc::adapt_encode_work_bound(0, n_streams)) return HC_ERR_ARG;
    Batch b{in, in_offs, in_lens, n_streams, out, out_offs, out_caps, out_lens, status, flags & HC_FLAG_DIFF};
    const hipError_t e = hc::adapt_encode_batch(b, widths, work, work_bytes, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? HC_OK : HC_ERR_DEVICE;
}

int hc_decompress_adapt_batch(const uint8_t *in, const uint64_t *in_offs, const uint64_t *in_lens,
                              uint32_t n_streams, uint8_t *out, const uint64_t *out_offs,
                              const uint64_t *out_caps, uint64_t *out_lens, int32_t *status, void *work,
                              uint64_t work_bytes, void *stream)
{
    if (n_streams == 0) return HC_OK;
    if (!in || !in_offs || !in_lens || !out || !out_offs || !out_caps || !out_lens || !status || !work)
        return HC_ERR_ARG;
    if (!aligned4(in) || !aligned4(out) || (reinterpret_cast<uintptr_t>(work) & 15u)) return HC_ERR_ARG;
    if (work_bytes < hc::adapt_decode_work_bound(0, 0, n_streams)) return HC_ERR_ARG;
    Batch b{in, in_offs, in_lens, n_streams, out, out_offs, out_caps, out_lens, status, 0};
    const hipError_t e = hc::adapt_decode_batch(b, work, work_bytes, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? HC_OK : HC_ERR_DEVICE;
}

const char *hc_version(void) { return "hcodec-mi355x 0.1 (gfx950)"; }

int hc_device_info(char *buf, uint64_t cap)
{
    int n = 0, dev = -1, rt = 0, drv = 0;
    hipError_t e = hipGetDeviceCount(&n);
    char arch[64] = "?";
    if (e == hipSuccess && n > 0) e = hipGetDevice(&dev);
    if (e == hipSuccess && n > 0) {
        hipDeviceProp_t prop;
        e = hipGetDeviceProperties(&prop, dev);
        if (e == hipSuccess) snprintf(arch, sizeof(arch), "%s", prop.gcnArchName);
    }
    (void)hipRuntimeGetVersion(&rt);
    (void)hipDriverGetVersion(&drv);
    if (buf && cap)
        snprintf(buf, cap, "devices=%d current=%d arch=%s runtime=%d driver=%d last=%s", n, dev, arch, rt, drv,
                 hipGetErrorString(e));
    return hc_device_ok();
}

int hc_device_ok(void)
{
    // the answer per device never changes: asked once per device (hipGetDeviceProperties is not
    // cheap next to a small single-buffer call)
    static std::atomic<int> known[64];  // 0 unknown, 1 gfx950, 2 other
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    if (dev < 64 && known[dev].load(std::memory_order_relaxed)) return known[dev].load(std::memory_order_relaxed) == 1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
    const int ok = strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
    if (dev < 64) known[dev].store(ok ? 1 : 2, std::memory_order_relaxed);
    return ok;
}

void hc_release_cached(void)
{
    FreeList &f = free_list();
    {
        std::lock_guard<std::mutex> lk(f.mu);
        for (int d = 0; d < 64; ++d) {
            for (auto &b : f.bufs[d]) (void)hipFree(b.first);
            f.bufs[d].clear();
            f.kept[d] = 0;
        }
    }
    hc::pipe_release();
}

}  // extern "C"
