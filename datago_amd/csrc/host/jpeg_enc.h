// jpeg_enc.h — host half of the JPEG re-encode (pre_encode_images,
// reference image_processing.rs:374-395): the header bytes (SOI .. SOS), the
// quality-scaled quantisation tables and the Annex K Huffman code tables the
// GPU kernels (dg_enc.hip) use.  image 0.25.9's JpegEncoder layout: APP0 JFIF
// 1.02, SOF0 (1x1 sampling), one DQT and one DHT segment per table, SOS.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../dg_types.h"

namespace dg {

// quality in [1, 100] -> natural-order tables (0 luma, 1 chroma), clamped to [1, 255]
void jpeg_enc_qtables(int quality, uint8_t q[2][64]);
// header bytes for a w x h image with ncomp (1 or 3) components
std::vector<uint8_t> jpeg_enc_header(uint32_t w, uint32_t h, int ncomp, int quality);
// code/length of every symbol of the four standard tables
void jpeg_enc_tables(EncTables &t);
// bytes the caller must provide for an encoded w x h x C image
uint64_t jpeg_enc_bound(uint32_t w, uint32_t h, uint32_t C);

}  // namespace dg
