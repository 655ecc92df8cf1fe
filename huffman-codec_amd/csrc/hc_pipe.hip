// hc_pipe.hip — host-buffer batches: many independent streams that live in host memory
// (files), pushed through the batched device coder in pipelined sub-batches (SURVEY.md §8f-1;
// the reference codes one file per process, main.cpp:202-220).
//
// Per sub-batch, on its own HIP stream: the inputs are packed into pinned staging (host
// memcpy), copied up, coded by the fused FGK kernels, then compacted on the device (each
// stream's bytes moved next to the previous stream's) so that only the produced bytes cross
// PCIe. Two slots alternate, so one sub-batch's kernels run while the previous one's results
// come back and are unpacked into the caller's buffers, and while the next one is staged.
// A stream whose output outgrows the sub-batch's device capacity guess reports the exact size
// and is coded again on its own.
#include <string.h>

#include <hipcub/hipcub.hpp>
#include <mutex>
#include <thread>
#include <vector>

#include "hc_internal.h"

namespace {

#define PIPE_CK(x)                                     \
    do {                                               \
        if ((x) != hipSuccess) return HC_ERR_DEVICE;   \
    } while (0)

constexpr uint64_t kAlign = 16;
uint64_t up16(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// copy(k) for k in [0, n) on up to 8 host threads when the bytes are many (staging into and out
// of pinned memory: one thread's memcpy would hold back the PCIe copies and the kernels)
template <class Copy>
void par_copy(uint32_t n, uint64_t bytes, Copy copy)
{
    const uint32_t hw = std::thread::hardware_concurrency();
    const uint32_t t = bytes < (32ull << 20) || n < 2 ? 1u : (hw < 2 ? 1u : (hw < 8 ? hw : 8u));
    if (t == 1) {
        for (uint32_t k = 0; k < n; ++k) copy(k);
        return;
    }
    std::vector<std::thread> th;
    for (uint32_t w = 0; w < t; ++w)
        th.emplace_back([&, w] {
            for (uint32_t k = (uint32_t)((uint64_t)n * w / t); k < (uint32_t)((uint64_t)n * (w + 1) / t); ++k) copy(k);
        });
    for (auto &x : th) x.join();
}

// length of the produced bytes that travel back (failed streams: none)
__global__ void kept_lengths(const uint64_t *lens, const int32_t *status, uint64_t *kept, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) kept[i] = status[i] == 0 ? lens[i] : 0;
}

// stream i's len[i] bytes from src + soffs[i] to dst + doffs[i]; one workgroup per stream per
// grid-stride step. The destination is packed back to back (any byte alignment): a byte head
// up to the next 16-byte boundary, then 16-byte aligned stores fed by unaligned 16-byte loads
// (global_load_dwordx4 takes any address on gfx950), then a byte tail.
typedef uint4 uint4_u __attribute__((aligned(1)));
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *src, const uint64_t *soffs, const uint64_t *lens,
                                                   uint32_t n, uint8_t *dst, const uint64_t *doffs)
{
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint8_t *s = src + soffs[i];
        uint8_t *d = dst + doffs[i];
        const uint64_t len = lens[i];
        uint64_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
        if (head > len) head = len;
        if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
        const uint64_t body = (len - head) / 16;
        const uint4_u *s16 = reinterpret_cast<const uint4_u *>(s + head);
        uint4 *d16 = reinterpret_cast<uint4 *>(d + head);
        for (uint64_t k = threadIdx.x; k < body; k += blockDim.x) {
            const uint4 v = {s16[k].x, s16[k].y, s16[k].z, s16[k].w};
            d16[k] = v;
        }
        const uint64_t t0 = head + body * 16;
        if (t0 + threadIdx.x < len) d[t0 + threadIdx.x] = s[t0 + threadIdx.x];
    }
}

template <class T>
struct Dev {
    T *p = nullptr;
    uint64_t cap = 0;
    ~Dev() { drop(); }
    void drop()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    hipError_t need(uint64_t n)
    {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const hipError_t e = hipMalloc(&p, (n ? n : 1) * sizeof(T));
        if (e == hipSuccess) cap = n;
        return e;
    }
};

template <class T>
struct Pinned {
    T *p = nullptr;
    uint64_t cap = 0;
    ~Pinned() { drop(); }
    void drop()
    {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    hipError_t need(uint64_t n)
    {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const hipError_t e = hipHostMalloc(&p, (n ? n : 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
};

// meta words per stream, uploaded / downloaded as one block: in_off, in_len, out_off, out_cap
// (up); out_len, status, kept offset (down)
struct Slot {
    hipStream_t st = nullptr;
    hipEvent_t meta_done = nullptr;
    Pinned<uint8_t> hin, hpacked;
    Pinned<uint64_t> hup, hdown;
    Dev<uint8_t> din, dout, dpacked, dtmp, dwork;
    Dev<uint64_t> dup, dlens, dkept, dat;
    Dev<int32_t> dstatus;
    uint32_t first = 0, count = 0;  // streams [first, first + count) of the call
    bool busy = false;
    ~Slot()
    {
        if (meta_done) (void)hipEventDestroy(meta_done);
        if (st) (void)hipStreamDestroy(st);
    }
    uint64_t device_bytes() const
    {
        return din.cap + dout.cap + dpacked.cap + dtmp.cap + dwork.cap + 8 * (dup.cap + dlens.cap + dkept.cap + dat.cap) +
               4 * dstatus.cap;
    }
    // free the buffers (the stream and event stay); the slot must be idle
    void release()
    {
        hin.drop();
        hpacked.drop();
        hup.drop();
        hdown.drop();
        din.drop();
        dout.drop();
        dpacked.drop();
        dtmp.drop();
        dwork.drop();
        dup.drop();
        dlens.drop();
        dkept.drop();
        dat.drop();
        dstatus.drop();
    }
};

// The two slots of one device, kept between calls (allocating and pinning a GiB per call cost
// more than the coding). One pool per device: a slot's stream and buffers belong to the device
// that was current when they were made.
struct Pool {
    std::mutex mu;
    Slot slots[2];
};
constexpr int kMaxDevices = 64;
std::mutex g_pools_mu;
Pool *g_pools[kMaxDevices];  // made on first use, never destroyed (the HIP runtime may be gone at exit)

Pool *pool_of(int dev)
{
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_pools_mu);
    if (!g_pools[dev]) g_pools[dev] = new Pool;
    return g_pools[dev];
}

struct Job {
    bool encode;
    bool adapt;              // -a streams: the batched adaptive device API (widths: encode only)
    const uint64_t *widths;
    uint32_t flags;
    const uint8_t *const *in;
    const uint64_t *in_lens;
    uint8_t *const *out;
    const uint64_t *out_caps;
    uint64_t *out_lens;
    int32_t *status;
    std::vector<uint64_t> dcap;  // device capacity per stream (a guess for decode)
};

// device capacity for stream i: encode — the input plus a quarter (FGK rarely expands data
// more; a stream that does reports its exact size and is redone); decode — the same idea
// against the header's symbol count (RLE expands 4 symbols to at most 258 bytes)
uint64_t guess_cap(const Job &j, uint32_t i)
{
    const uint64_t n = j.in_lens[i];
    uint64_t c;
    if (j.encode) {
        c = j.adapt ? hc_compress_bound(n, 1) : n + n / 4 + 4096;
    } else {
        uint64_t count = 0;
        if (n >= 9)
            for (int b = 7; b >= 0; --b) count = (count << 8) | j.in[i][b];
        const uint64_t most = count * 65 + 8;
        c = n * 8 > 65536 ? n * 8 : 65536;
        if (c > most) c = most;
    }
    return c < j.out_caps[i] ? c : j.out_caps[i];
}

int launch(Job &j, Slot &s)
{
    const uint32_t n = s.count;
    uint64_t in_bytes = 0, out_bytes = 0;
    for (uint32_t k = 0; k < n; ++k) {
        in_bytes += up16(j.in_lens[s.first + k]);
        out_bytes += up16(j.dcap[s.first + k]);
    }
    const uint64_t cols = j.adapt && j.encode ? 5 : 4;  // + the widths column
    PIPE_CK(s.hin.need(in_bytes));
    PIPE_CK(s.hup.need(cols * n));
    PIPE_CK(s.hdown.need(3ull * n + 1));
    PIPE_CK(s.din.need(in_bytes));
    PIPE_CK(s.dout.need(out_bytes));
    PIPE_CK(s.dpacked.need(out_bytes));
    PIPE_CK(s.dup.need(cols * n));
    PIPE_CK(s.dlens.need(n));
    PIPE_CK(s.dkept.need(n));
    PIPE_CK(s.dat.need(n + 1));
    PIPE_CK(s.dstatus.need(n));
    // stage: inputs packed at 16-byte aligned offsets, meta columns
    uint64_t *up = s.hup.p;
    uint64_t io = 0, oo = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t i = s.first + k;
        const uint64_t len = j.in_lens[i];
        up[k] = io;
        up[n + k] = len;
        up[2 * n + k] = oo;
        up[3 * n + k] = j.dcap[i];
        if (cols == 5) up[4 * n + k] = j.widths[i];
        io += up16(len);
        oo += up16(j.dcap[i]);
    }
    par_copy(n, in_bytes, [&](uint32_t k) {
        if (up[n + k]) memcpy(s.hin.p + up[k], j.in[s.first + k], up[n + k]);
    });
    PIPE_CK(hipMemcpyAsync(s.din.p, s.hin.p, in_bytes, hipMemcpyHostToDevice, s.st));
    PIPE_CK(hipMemcpyAsync(s.dup.p, up, cols * n * sizeof(uint64_t), hipMemcpyHostToDevice, s.st));
    const uint64_t *d = s.dup.p;
    hc::Batch b{s.din.p, d, d + n, n, s.dout.p, d + 2 * n, d + 3 * n, s.dlens.p, s.dstatus.p, j.flags};
    if (j.adapt) {  // workspace of the adaptive stages, sized for this sub-batch
        const uint64_t wb = j.encode ? hc::adapt_encode_work_bound(in_bytes, n)
                                     : hc::adapt_decode_work_bound(in_bytes, out_bytes, n);
        PIPE_CK(s.dwork.need(wb));
        if (j.encode)
            PIPE_CK(hc::adapt_encode_batch(b, d + 4 * n, s.dwork.p, s.dwork.cap, s.st));
        else
            PIPE_CK(hc::adapt_decode_batch(b, s.dwork.p, s.dwork.cap, s.st));
    } else if (j.encode) {
        PIPE_CK(hc::launch_encode(b, (j.flags & HC_FLAG_DIFF) ? hc::SRC_RAW_DIFF : hc::SRC_RAW, s.st));
    } else {
        PIPE_CK(hc::launch_decode(b, hc::DST_RAW, s.st));
    }
    // compaction: kept lengths, their exclusive scan (+ total), the copy
    kept_lengths<<<(n + 255) / 256, 256, 0, s.st>>>(s.dlens.p, s.dstatus.p, s.dkept.p, n);
    size_t tb = 0;
    PIPE_CK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, s.dkept.p, s.dat.p, (int)n, s.st));
    PIPE_CK(s.dtmp.need(tb));
    PIPE_CK(hipcub::DeviceScan::ExclusiveSum(s.dtmp.p, tb, s.dkept.p, s.dat.p, (int)n, s.st));
    pack_kernel<<<n < 65535 ? n : 65535, 256, 0, s.st>>>(s.dout.p, d + 2 * n, s.dkept.p, n, s.dpacked.p, s.dat.p);
    PIPE_CK(hipGetLastError());
    PIPE_CK(hipMemcpyAsync(s.hdown.p, s.dlens.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s.st));
    PIPE_CK(hipMemcpyAsync(s.hdown.p + n, s.dat.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s.st));
    PIPE_CK(hipMemcpyAsync(s.hdown.p + 2 * n, s.dstatus.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, s.st));
    PIPE_CK(hipEventRecord(s.meta_done, s.st));
    s.busy = true;
    return HC_OK;
}

// results of slot s: wait for its meta, bring the packed bytes, unpack into the caller's buffers
int finish(Job &j, Slot &s, std::vector<uint32_t> &redo)
{
    const uint32_t n = s.count;
    PIPE_CK(hipEventSynchronize(s.meta_done));
    const uint64_t *lens = s.hdown.p, *at = s.hdown.p + n;
    const int32_t *st = reinterpret_cast<const int32_t *>(s.hdown.p + 2 * n);
    uint64_t total = 0;
    for (uint32_t k = 0; k < n; ++k)
        if (st[k] == 0) total = at[k] + lens[k];
    PIPE_CK(s.hpacked.need(total));
    if (total) {
        PIPE_CK(hipMemcpyAsync(s.hpacked.p, s.dpacked.p, total, hipMemcpyDeviceToHost, s.st));
        PIPE_CK(hipStreamSynchronize(s.st));
    }
    par_copy(n, total, [&](uint32_t k) {
        if (st[k] == 0 && lens[k]) memcpy(j.out[s.first + k], s.hpacked.p + at[k], lens[k]);
    });
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t i = s.first + k;
        j.out_lens[i] = lens[k];
        j.status[i] = st[k];
        if (st[k] == 0) {
        } else if (st[k] == HC_ERR_CAPACITY && j.dcap[i] < j.out_caps[i]) {
            // the guess was short: code it again with what it needs (or all the caller has)
            j.dcap[i] = lens[k] < j.out_caps[i] ? lens[k] : j.out_caps[i];
            redo.push_back(i);
        }
    }
    s.busy = false;
    return HC_OK;
}

uint64_t env_u64(const char *name, uint64_t dflt)
{
    const char *v = getenv(name);
    if (!v || !*v) return dflt;
    const uint64_t x = strtoull(v, nullptr, 0);
    return x ? x : dflt;
}

int run_slots(Job &j, uint32_t n, Slot *slots);

int run(Job &j, uint32_t n)
{
    if (n == 0) return HC_OK;
    if (!j.in || !j.in_lens || !j.out || !j.out_caps || !j.out_lens || !j.status) return HC_ERR_ARG;
    for (uint32_t i = 0; i < n; ++i)
        if ((!j.in[i] && j.in_lens[i]) || (!j.out[i] && j.out_caps[i])) return HC_ERR_ARG;
    if (!hc_device_ok()) return HC_ERR_DEVICE;
    j.dcap.resize(n);
    for (uint32_t i = 0; i < n; ++i) j.dcap[i] = guess_cap(j, i);
    // the current device's two slots (kept between calls); a concurrent call on the same device
    // gets slots of its own, freed when it returns
    int dev = -1;
    PIPE_CK(hipGetDevice(&dev));
    Pool *const pool = pool_of(dev);
    std::unique_lock<std::mutex> lk;
    if (pool) lk = std::unique_lock<std::mutex>(pool->mu, std::try_to_lock);
    Slot local[2];
    Slot *const slots = lk.owns_lock() ? pool->slots : local;
    const int rc = run_slots(j, n, slots);
    // the kept slots give back what is above HC_PIPE_KEEP_BYTES (default 8 GiB of device
    // buffers; e.g. after a large adaptive decode) -- their work is done once run_slots returns
    if (lk.owns_lock()) {
        const uint64_t keep = env_u64("HC_PIPE_KEEP_BYTES", 8ull << 30);
        if (slots[0].device_bytes() + slots[1].device_bytes() > keep)
            for (int k = 0; k < 2; ++k) {
                (void)hipStreamSynchronize(slots[k].st);
                slots[k].release();
            }
    }
    return rc;
}

int run_slots(Job &j, uint32_t n, Slot *slots)
{
    // sub-batch limits: input bytes and streams per slot (HC_PIPE_BYTES / HC_PIPE_STREAMS)
    const uint64_t max_bytes = env_u64("HC_PIPE_BYTES", 1ull << 30);
    const uint64_t max_streams = env_u64("HC_PIPE_STREAMS", 8192);
    for (int k = 0; k < 2; ++k) {
        Slot &s = slots[k];
        s.busy = false;
        if (!s.st) PIPE_CK(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
        if (!s.meta_done) PIPE_CK(hipEventCreateWithFlags(&s.meta_done, hipEventDisableTiming));
        PIPE_CK(hipStreamSynchronize(s.st));  // (a call that failed may have left work queued)
    }
    std::vector<uint32_t> order(n), redo;
    for (uint32_t i = 0; i < n; ++i) order[i] = i;
    for (int pass = 0; pass < 2 && !order.empty(); ++pass) {
        // pass 1 codes the streams whose capacity guess fell short, one per sub-batch entry
        std::vector<uint32_t> cur;
        cur.swap(order);
        uint32_t pos = 0, turn = 0;
        while (pos < cur.size()) {
            Slot &s = slots[turn++ & 1];
            if (s.busy) {
                const int rc = finish(j, s, redo);
                if (rc) return rc;
            }
            // streams of one sub-batch must be contiguous in the job: pass 0 is in order; in
            // pass 1 each stream forms its own sub-batch
            uint64_t bytes = 0;
            uint32_t cnt = 0;
            if (pass == 0) {
                while (pos + cnt < cur.size() && cnt < max_streams &&
                       (cnt == 0 || bytes + j.in_lens[cur[pos + cnt]] <= max_bytes)) {
                    bytes += j.in_lens[cur[pos + cnt]];
                    ++cnt;
                }
            } else {
                cnt = 1;
            }
            s.first = cur[pos];
            s.count = cnt;
            pos += cnt;
            const int rc = launch(j, s);
            if (rc) return rc;
        }
        for (int k = 0; k < 2; ++k) {
            Slot &s = slots[turn++ & 1];
            if (s.busy) {
                const int rc = finish(j, s, redo);
                if (rc) return rc;
            }
        }
        order.swap(redo);
        redo.clear();
    }
    return HC_OK;
}

}  // namespace

namespace hc {
void pipe_release()
{
    std::lock_guard<std::mutex> lk(g_pools_mu);
    for (Pool *p : g_pools) {
        if (!p) continue;
        std::unique_lock<std::mutex> pl(p->mu, std::try_to_lock);
        if (!pl.owns_lock()) continue;  // a call is using it
        for (Slot &s : p->slots) {
            if (s.st) (void)hipStreamSynchronize(s.st);
            s.release();
        }
    }
}
}  // namespace hc

extern "C" {

int hc_compress_host_batch(const uint8_t *const *in, const uint64_t *in_lens, uint32_t n_streams,
                           uint32_t flags, uint8_t *const *out, const uint64_t *out_caps,
                           uint64_t *out_lens, int32_t *status)
{
    if (flags & ~HC_FLAG_DIFF) return HC_ERR_ARG;
    Job j{true, false, nullptr, flags, in, in_lens, out, out_caps, out_lens, status, {}};
    return run(j, n_streams);
}

int hc_compress_adapt_host_batch(const uint8_t *const *in, const uint64_t *in_lens, const uint64_t *widths,
                                 uint32_t n_streams, uint32_t flags, uint8_t *const *out, const uint64_t *out_caps,
                                 uint64_t *out_lens, int32_t *status)
{
    if ((flags & ~HC_FLAG_DIFF) || (n_streams && !widths)) return HC_ERR_ARG;
    Job j{true, true, widths, flags, in, in_lens, out, out_caps, out_lens, status, {}};
    return run(j, n_streams);
}

int hc_pack_batch(const uint8_t *in, const uint64_t *in_offs, const uint64_t *lens, uint32_t n_streams,
                  uint8_t *out, const uint64_t *out_offs, void *stream)
{
    if (n_streams == 0) return HC_OK;
    if (!in || !in_offs || !lens || !out || !out_offs) return HC_ERR_ARG;
    pack_kernel<<<n_streams < 65535 ? n_streams : 65535, 256, 0, static_cast<hipStream_t>(stream)>>>(
        in, in_offs, lens, n_streams, out, out_offs);
    return hipGetLastError() == hipSuccess ? HC_OK : HC_ERR_DEVICE;
}

int hc_decompress_host_batch(const uint8_t *const *in, const uint64_t *in_lens, uint32_t n_streams,
                             uint8_t *const *out, const uint64_t *out_caps, uint64_t *out_lens,
                             int32_t *status)
{
    if (n_streams && (!in || !in_lens)) return HC_ERR_ARG;
    // adaptive streams (flags bit 6) and the rest go through their own device paths, each as
    // one job over the streams of its kind (gathered, results scattered back)
    std::vector<uint32_t> ids[2];
    for (uint32_t i = 0; i < n_streams; ++i) {
        const bool a = in_lens[i] >= 9 && in[i] && (in[i][8] & HC_FLAG_ADAPT);
        ids[a].push_back(i);
    }
    for (int a = 0; a < 2; ++a) {
        const std::vector<uint32_t> &id = ids[a];
        if (id.empty()) continue;
        if (id.size() == n_streams) {
            Job j{false, a == 1, nullptr, 0, in, in_lens, out, out_caps, out_lens, status, {}};
            return run(j, n_streams);
        }
        const size_t m = id.size();
        std::vector<const uint8_t *> ip(m);
        std::vector<uint8_t *> op(m);
        std::vector<uint64_t> il(m), oc(m), ol(m, 0);
        std::vector<int32_t> st(m, 0);
        for (size_t k = 0; k < m; ++k) {
            ip[k] = in[id[k]];
            il[k] = in_lens[id[k]];
            op[k] = out ? out[id[k]] : nullptr;
            oc[k] = out_caps ? out_caps[id[k]] : 0;
        }
        Job j{false, a == 1, nullptr, 0, ip.data(), il.data(), op.data(), oc.data(), ol.data(), st.data(), {}};
        const int rc = run(j, (uint32_t)m);
        if (rc) return rc;
        for (size_t k = 0; k < m; ++k) {
            if (out_lens) out_lens[id[k]] = ol[k];
            if (status) status[id[k]] = st[k];
        }
    }
    return HC_OK;
}

}  // extern "C"
