// hc_cli.cpp — `huffman-codec`, the drop-in command line of the MI355X codec.
//
// Same contract as the reference's src/main.cpp:152-221: getopt(":cdmai:o:w:h"), -c default,
// last of -c/-d wins, -w parsed by std::stoull (default 512; a non-numeric value throws and
// aborts exactly like the reference), -o default b.out, the same help text, error messages and
// exit codes 1-15, and the stderr line "writing N bytes to F". Compression and decompression
// run on the GPU through include/hcodec.h.
//
// HC_CLI_TIMES=1 (bench.py's C1 line): after the normal output, one extra stderr line with the
// time of each phase inside the process (read, HIP start-up, coding, write, ms), so that the
// per-file cost can be split from the process start the caller measures around it.
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "hc_messages.h"
#include "hcodec.h"

namespace {

const char *const kHelp =
    "USAGE:\n"
    "  huffman-codec [-cm] -i IFILE [-o OFILE]\n"
    "  huffman-codec [-cm] -a [-w WIDTH] -i IFILE [-o OFILE]\n"
    "  huffman-codec -d -i IFILE [-o OFILE] | -h\n"
    "\n"
    "OPTION:\n"
    "  -c/-d  perform compression/decompression\n"
    "  -m     use differential model for preprocessing\n"
    "  -a     use adaptive block RLE (default: RLE)\n"
    "  -w     width of 2D data (default: 512)\n"
    "  -i     input file path\n"
    "  -o     output file path (default: b.out)\n"
    "  -h     show this help\n";

void error_hint(const char *msg)  // main.cpp:147-149
{
    std::cerr << msg << "try 'huffman-codec -h' for more information\n";
}

double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

int main(int argc, char *argv[])
{
    bool compress = true, use_diff = false, use_adapt = false;
    std::string ifp, ofp = "b.out";
    uint64_t width = 512;

    int opt;
    while ((opt = getopt(argc, argv, ":cdmai:o:w:h")) != -1) {
        switch (opt) {
        case 'c': compress = true; break;
        case 'd': compress = false; break;
        case 'm': use_diff = true; break;
        case 'a': use_adapt = true; break;
        case 'i': ifp = optarg; break;
        case 'o': ofp = optarg; break;
        case 'w': width = std::stoull(optarg); break;  // throws like main.cpp:176
        case 'h': std::cout << kHelp; return 0;
        case ':': error_hint("ERROR: missing additional argument\n"); return 1;
        case '?': error_hint("ERROR: unrecognized option used\n"); return 2;
        }
    }
    if (ifp.empty()) {
        error_hint("ERROR: no input file path provided\n");
        return 3;
    }
    if (compress && width == 0) {
        error_hint("ERROR: invalid 2D data width\n");
        return 4;
    }
    const char *times_env = std::getenv("HC_CLI_TIMES");
    const bool times = times_env && times_env[0] == '1';
    double t_read = 0, t_init = 0, t_code = 0, t_again = 0;
    auto t0 = std::chrono::steady_clock::now();
    std::ifstream ifs(ifp, std::ios::in | std::ios::binary);
    if (ifs.fail()) {
        std::cerr << "ERROR: given input file does not exist\n";
        return 5;
    }
    const std::vector<uint8_t> in((std::istreambuf_iterator<char>(ifs)), std::istreambuf_iterator<char>());
    ifs.close();
    if (times) {
        t_read = ms_since(t0);
        t0 = std::chrono::steady_clock::now();
        (void)hc_device_ok();  // HIP start-up apart from the coding (otherwise the first call's)
        t_init = ms_since(t0);
        t0 = std::chrono::steady_clock::now();
    }

    std::vector<uint8_t> out;
    int st;
    if (compress) {
        out.resize(hc_compress_bound(in.size(), use_adapt ? 1 : 0));
        uint64_t len = 0;
        st = hc_compress(in.data(), in.size(), use_diff, use_adapt, width, out.data(), out.size(), &len);
        out.resize(st == HC_OK ? len : 0);
    } else {
        uint8_t *p = nullptr;
        uint64_t len = 0;
        st = hc_decompress_alloc(in.data(), in.size(), &p, &len);
        if (st == HC_OK) out.assign(p, p + len);
        hc_free(p);
    }
    if (times) {
        t_code = ms_since(t0);
        // the same call once more in this process: without the first call's one-time costs (the
        // code objects' load at the first launch, the device buffers' first allocation), i.e. the
        // copies in and out plus the kernels
        t0 = std::chrono::steady_clock::now();
        std::vector<uint8_t> again(compress ? hc_compress_bound(in.size(), use_adapt ? 1 : 0) : 0);
        uint64_t len2 = 0;
        uint8_t *p2 = nullptr;
        if (compress) (void)hc_compress(in.data(), in.size(), use_diff, use_adapt, width, again.data(), again.size(), &len2);
        else if (hc_decompress_alloc(in.data(), in.size(), &p2, &len2) == HC_OK) hc_free(p2);
        t_again = ms_since(t0);
        t0 = std::chrono::steady_clock::now();
    }
    if (st != HC_OK) {
        std::cerr << hc_status_message(st);
        return st;
    }

    std::cerr << "writing " << out.size() << " bytes to " << ofp << "\n";  // main.cpp:218
    std::ofstream ofs(ofp, std::ios::out | std::ios::binary);                // main.cpp:132-144
    if (ofs.fail()) {
        std::cerr << "ERROR: cannot write to " << ofp << " output file\n";
        return 7;
    }
    ofs.write(reinterpret_cast<const char *>(out.data()), (std::streamsize)out.size());
    if (times) {
        ofs.close();
        std::cerr << "hc-times read_ms=" << t_read << " hip_init_ms=" << t_init << " code_ms=" << t_code
                  << " write_ms=" << ms_since(t0) << " code_again_ms=" << t_again << "\n";
    }
    return 0;
}
