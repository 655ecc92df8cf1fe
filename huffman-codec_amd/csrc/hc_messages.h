// hc_messages.h — the reference's error messages for the statuses its library exits with
// (transform.cpp, headers.cpp, main.cpp), shared by both command lines.
#pragma once

#include "hcodec.h"

// the reference's messages for the statuses its library exits with
inline const char *hc_status_message(int st)
{
    switch (st) {
    case HC_ERR_MATRIX_SIZE: return "ERROR: invalid size of input 2D data detected\n";
    case HC_ERR_HEADER: return "ERROR: invalid or missing Huffman coding header\n";
    case HC_ERR_HUFFMAN: return "ERROR: invalid Huffman coding file contents\n";
    case HC_ERR_ADAPT_HEADER: return "ERROR: invalid or missing adaptive block RLE header\n";
    case HC_ERR_ADAPT_DIRS: return "ERROR: invalid adaptive block RLE header\n";
    case HC_ERR_DIMS: return "ERROR: too small 2D data dimensions\n";
    case HC_ERR_BLOCK_DATA: return "ERROR: invalid adaptive block RLE file contents\n";
    case HC_ERR_BLOCK_EOF: return "ERROR: unexpected end of adaptive block RLE data\n";
    case HC_ERR_LEFTOVER: return "ERROR: leftover data of adaptive block RLE detected\n";
    case HC_ERR_BLOCK_SIZE: return "ERROR: invalid adaptive block RLE block size\n";
    case HC_ERR_TOO_LARGE: return "ERROR: adaptive block RLE matrix too large\n";
    case HC_ERR_UNSUPPORTED: return "ERROR: stream exceeds the device coder's limits\n";
    case HC_ERR_DEVICE: return "ERROR: no usable gfx950 GPU (HIP runtime error)\n";
    default: return "ERROR: codec failure\n";
    }
}

