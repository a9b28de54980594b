// png_header.h — host-side PNG chunk walker (signature .. IEND), no pixel work.
//
// Replaces the header half of `image::load_from_memory` / `ImageReader::decode`
// for PNG (reference worker_files.rs:14-16, worker_wds.rs:45; image 0.25.9 ->
// png 0.18.0 with Transformations::EXPAND).  It validates IHDR, collects PLTE /
// tRNS (folded into a 256-entry RGBA palette or a gray/RGB key) and the
// positions of the IDAT payloads; inflate, unfiltering and expansion run on
// the GPU (kernels.hip, k_png_*).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace dg {

enum PngStatus { PH_OK = 0, PH_UNSUPPORTED = 1, PH_CORRUPT = 2 };

struct PngHeader {
  int status = PH_CORRUPT;
  const char *why = "";
  uint32_t width = 0, height = 0;
  int depth = 0, ctype = 0, interlace = 0;
  int spp = 0;           // samples per pixel in the file (1 gray/palette, 2 LA, 3 RGB, 4 RGBA)
  int out_c = 0;         // channels after EXPAND: L8 1, La8 2, Rgb8 3, Rgba8 4
  int bpp = 1;           // filter unit in bytes (PNG spec 9.2)
  uint32_t rowbytes = 0; // bytes per unfiltered scanline (without the filter byte)
  uint8_t pal[256][4];   // palette as RGBA (tRNS alpha, 255 default; black past PLTE)
  int npal = 0;
  int has_trns = 0;
  uint16_t trns[3] = {0, 0, 0};  // gray / RGB transparency key (file sample values)
  std::vector<uint32_t> idat_off, idat_len;  // IDAT payload positions in the file
  uint64_t zlen = 0;     // total zlib bytes
  uint64_t rawlen = 0;   // inflated bytes: filtered rows (+1 filter byte each) of the image or of its 7 Adam7 passes
  uint64_t unflen = 0;   // unfiltered bytes at 16-byte row strides (per pass when interlaced)
};

bool is_png(const uint8_t *d, size_t n);
// PNG re-encode (dg_penc.hip): signature + IHDR chunk (8-bit, C = 1/2/3/4
// channels -> colour type 0/4/2/6, no interlace) and the output size bound.
std::vector<uint8_t> png_enc_header(uint32_t w, uint32_t h, uint32_t C);
uint64_t png_enc_bound(uint32_t w, uint32_t h, uint32_t C);
// Walks every chunk header (reads 8 bytes per chunk plus IHDR/PLTE/tRNS payloads).
void parse_png_header(const uint8_t *d, size_t n, PngHeader &h);

}  // namespace dg
