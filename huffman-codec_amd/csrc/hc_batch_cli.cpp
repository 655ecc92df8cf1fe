// hc_batch_cli.cpp — `huffman-codec-batch`: many files per process through the pipelined
// host-batch API of include/hcodec.h (the reference codes one file per
// process, main.cpp:202-220). Each output is byte-identical to what `huffman-codec` (and the
// reference) writes for that file alone.
//
//   huffman-codec-batch [-c | -d] [-m] [-a [-w WIDTH]] [-o OUTDIR] [-j THREADS] FILE...
//
// Compression writes FILE.huf, decompression FILE without its .huf suffix (else FILE.out);
// with -o into OUTDIR under the same base name. Files are read and written by a pool of
// THREADS host threads (default 8). All files go through the pipelined host-batch API in one
// call: hc_compress_host_batch, hc_compress_adapt_host_batch (-a: one matrix of width WIDTH per
// file) or hc_decompress_host_batch (any mix of adaptive and plain streams). A file that fails reports
// "FILE: <the reference's message>"; the exit code is the first failing status (0: all ok).
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

#include "hc_messages.h"
#include "hcodec.h"

namespace {

const char *const kHelp =
    "USAGE:\n"
    "  huffman-codec-batch [-cm] [-o OUTDIR] [-j THREADS] FILE...\n"
    "  huffman-codec-batch [-cm] -a [-w WIDTH] [-o OUTDIR] [-j THREADS] FILE...\n"
    "  huffman-codec-batch -d [-o OUTDIR] [-j THREADS] FILE... | -h\n"
    "\n"
    "OPTION:\n"
    "  -c/-d  perform compression/decompression\n"
    "  -m     use differential model for preprocessing\n"
    "  -a     use adaptive block RLE (default: RLE)\n"
    "  -w     width of 2D data (default: 512)\n"
    "  -o     output directory (default: next to each input)\n"
    "  -j     file I/O threads (default: 8)\n"
    "  -h     show this help\n"
    "OUTPUT:\n"
    "  -c: FILE.huf   -d: FILE without .huf (else FILE.out)\n";

std::string base_name(const std::string &p)
{
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? p : p.substr(k + 1);
}

std::string out_path(const std::string &in, bool compress, const std::string &dir)
{
    std::string name = dir.empty() ? in : dir + "/" + base_name(in);
    if (compress) return name + ".huf";
    if (name.size() > 4 && name.compare(name.size() - 4, 4, ".huf") == 0) return name.substr(0, name.size() - 4);
    return name + ".out";
}

// run f(i) for i in [0, n) on `threads` host threads
template <class F>
void parallel(size_t n, unsigned threads, F &&f)
{
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < std::max(1u, threads); ++t)
        pool.emplace_back([&] {
            for (size_t i; (i = next++) < n;) f(i);
        });
    for (auto &th : pool) th.join();
}

}  // namespace

int main(int argc, char *argv[])
{
    bool compress = true, use_diff = false, use_adapt = false;
    std::string dir;
    uint64_t width = 512;
    unsigned threads = 8;
    int opt;
    while ((opt = getopt(argc, argv, ":cdmaw:o:j:h")) != -1) {
        switch (opt) {
        case 'c': compress = true; break;
        case 'd': compress = false; break;
        case 'm': use_diff = true; break;
        case 'a': use_adapt = true; break;
        case 'w': width = std::stoull(optarg); break;
        case 'o': dir = optarg; break;
        case 'j': threads = (unsigned)std::stoul(optarg); break;
        case 'h': std::cout << kHelp; return 0;
        case ':': std::cerr << "ERROR: missing additional argument\n"; return 1;
        case '?': std::cerr << "ERROR: unrecognized option used\n"; return 2;
        }
    }
    std::vector<std::string> files(argv + optind, argv + argc);
    if (files.empty()) {
        std::cerr << "ERROR: no input file path provided\n";
        return 3;
    }
    if (compress && width == 0) {
        std::cerr << "ERROR: invalid 2D data width\n";
        return 4;
    }
    const size_t n = files.size();
    std::vector<std::vector<uint8_t>> in(n), out(n);
    std::vector<int> status(n, 0);
    parallel(n, threads, [&](size_t i) {
        std::ifstream ifs(files[i], std::ios::in | std::ios::binary);
        if (ifs.fail()) {
            status[i] = 5;  // main.cpp:205-208
            return;
        }
        in[i].assign(std::istreambuf_iterator<char>(ifs), std::istreambuf_iterator<char>());
    });

    if (compress) {  // -a: one matrix of width `width` per file
        std::vector<const uint8_t *> ip(n);
        std::vector<uint8_t *> op(n);
        std::vector<uint64_t> il(n), oc(n), ol(n), wd(n, width);
        std::vector<int32_t> st(n, 0);
        for (size_t i = 0; i < n; ++i) {
            ip[i] = in[i].data();
            il[i] = status[i] ? 0 : in[i].size();
            out[i].resize(hc_compress_bound(il[i], use_adapt));
            op[i] = out[i].data();
            oc[i] = out[i].size();
        }
        const uint32_t fl = use_diff ? HC_FLAG_DIFF : 0;
        const int rc = use_adapt ? hc_compress_adapt_host_batch(ip.data(), il.data(), wd.data(), (uint32_t)n, fl,
                                                                op.data(), oc.data(), ol.data(), st.data())
                                 : hc_compress_host_batch(ip.data(), il.data(), (uint32_t)n, fl, op.data(), oc.data(),
                                                          ol.data(), st.data());
        if (rc) {
            std::cerr << hc_status_message(rc);
            return rc;
        }
        for (size_t i = 0; i < n; ++i) {
            if (!status[i]) status[i] = st[i];
            out[i].resize(status[i] ? 0 : ol[i]);
        }
    } else {
        // one batch (adaptive and plain streams alike), whose output sizes are unknown up
        // front: a guess, then the exact size for those that report it
        std::vector<size_t> batch;
        for (size_t i = 0; i < n; ++i)
            if (!status[i]) batch.push_back(i);
        for (int pass = 0; pass < 2 && !batch.empty(); ++pass) {
            const size_t m = batch.size();
            std::vector<const uint8_t *> ip(m);
            std::vector<uint8_t *> op(m);
            std::vector<uint64_t> il(m), oc(m), ol(m);
            std::vector<int32_t> st(m, 0);
            for (size_t k = 0; k < m; ++k) {
                const size_t i = batch[k];
                ip[k] = in[i].data();
                il[k] = in[i].size();
                if (pass == 0) out[i].resize(std::max<uint64_t>(il[k] * 8, 65536));
                op[k] = out[i].data();
                oc[k] = out[i].size();
            }
            const int rc = hc_decompress_host_batch(ip.data(), il.data(), (uint32_t)m, op.data(), oc.data(), ol.data(),
                                                    st.data());
            if (rc) {
                std::cerr << hc_status_message(rc);
                return rc;
            }
            std::vector<size_t> again;
            for (size_t k = 0; k < m; ++k) {
                const size_t i = batch[k];
                if (st[k] == HC_ERR_CAPACITY && pass == 0) {
                    out[i].resize(ol[k]);
                    again.push_back(i);
                    continue;
                }
                status[i] = st[k];
                out[i].resize(st[k] ? 0 : ol[k]);
            }
            batch.swap(again);
        }
    }

    std::atomic<int> first_fail{0};
    std::vector<std::string> msgs(n);
    parallel(n, threads, [&](size_t i) {
        if (status[i] == 5) {
            msgs[i] = files[i] + ": ERROR: given input file does not exist\n";
            return;
        }
        if (status[i]) {
            msgs[i] = files[i] + ": " + hc_status_message(status[i]);
            return;
        }
        const std::string op = out_path(files[i], compress, dir);
        std::ofstream ofs(op, std::ios::out | std::ios::binary);
        if (ofs.fail()) {
            status[i] = 7;  // main.cpp:132-144
            msgs[i] = files[i] + ": ERROR: cannot write to " + op + " output file\n";
            return;
        }
        ofs.write(reinterpret_cast<const char *>(out[i].data()), (std::streamsize)out[i].size());
    });
    uint64_t in_bytes = 0, out_bytes = 0, ok = 0;
    for (size_t i = 0; i < n; ++i) {
        if (status[i]) {
            std::cerr << msgs[i];
            int z = 0;
            first_fail.compare_exchange_strong(z, status[i]);
            continue;
        }
        ++ok;
        in_bytes += in[i].size();
        out_bytes += out[i].size();
    }
    std::cerr << "coded " << ok << " of " << n << " files, " << in_bytes << " -> " << out_bytes << " bytes\n";
    return first_fail.load();
}
