// jpeg_header.h — host-side JPEG marker parser (SOI..SOS), header only.
//
// Replaces the header half of `ImageReader::with_guessed_format().decode()`
// (reference worker_files.rs:14-16; image 0.25.9 -> zune-jpeg 0.5.12): it
// validates the stream, decides whether the GPU path can decode it (baseline /
// extended sequential Huffman with a single interleaved scan, or progressive
// Huffman; 8-bit, 1 or 3 components, h2v1/h2v2/1x1 chroma) and gathers
// everything the kernels need.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../dg_types.h"

namespace dg {

struct HuffSpec {
  bool present = false;
  uint8_t bits[17] = {0};
  uint8_t vals[256] = {0};
  int nvals = 0;
};

// One scan of a progressive JPEG (T.81 G.1.2): its components, spectral
// band [ss, se], successive-approximation bits ah/al, the Huffman tables in
// force when it starts and its entropy-coded bytes [off, end).
struct JpegScan {
  int ns = 0;
  int comp[4] = {0, 0, 0, 0};
  int dc_tab[4] = {-1, -1, -1, -1};  // index into JpegHeader::tables (DC first scans)
  int ac_tab = -1;                    // AC scans (ns == 1)
  int ss = 0, se = 0, ah = 0, al = 0;
  int restart = 0;
  size_t off = 0, end = 0;
};

struct JpegComponent {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
};

enum JpegStatus { JH_OK = 0, JH_UNSUPPORTED = 1, JH_CORRUPT = 2 };

struct JpegHeader {
  int status = JH_CORRUPT;
  const char *why = "";
  int sof = 0;  // marker code (0xC0..)
  int precision = 8;
  uint32_t width = 0, height = 0;
  int ncomp = 0;
  JpegComponent comp[4];
  bool progressive = false, arithmetic = false, lossless = false;
  bool incomplete_refinement = false;  // progressive: DC or AC 1..9 not fully refined (libjpeg would smooth blocks)
  int restart = 0;
  bool jfif = false, adobe = false;
  int adobe_transform = -1;
  uint16_t q[4][64];  // natural order
  bool qpresent[4] = {false, false, false, false};
  HuffSpec dc[4], ac[4];
  int scan_ncomp = 0;
  int scan_comp[4] = {0, 0, 0, 0};
  size_t scan_off = 0;   // first entropy-coded byte
  size_t scan_end = 0;   // end of entropy data (EOI position if found at the end)
  int hmax = 1, vmax = 1;
  int colorspace = CS_YCC;
  // progressive files: every scan, and snapshots of the Huffman tables they use
  std::vector<JpegScan> scans;
  std::vector<HuffSpec> tables;
};

// Parse up to (and including) the SOS header.  Only touches bytes before the
// entropy-coded segment plus the last two bytes (EOI check).
void parse_jpeg_header(const uint8_t *d, size_t n, JpegHeader &h);

// Canonical Huffman code -> GPU lookup table (T.81 Annex C).  Returns false
// for an over-subscribed code.
bool build_huff_table(const HuffSpec &spec, HuffTable &out);

bool is_jpeg(const uint8_t *d, size_t n);
// Marker walk up to the first SOFn: true for SOF2 (progressive, Huffman).
bool jpeg_sniff_progressive(const uint8_t *d, size_t n);
bool is_png(const uint8_t *d, size_t n);

}  // namespace dg
