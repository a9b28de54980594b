// jpeg_enc.cpp — see jpeg_enc.h.
#include "jpeg_enc.h"

#include <string.h>

namespace dg {

namespace {
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// ITU-T T.81 Annex K.1 (natural order)
const uint8_t kLumaQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                            14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                            18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                            49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChromaQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                              24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// Annex K.3 Huffman tables
const uint8_t kDcLumaBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcChromaBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumaBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumaVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChromaBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChromaVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

void segment(std::vector<uint8_t> &o, uint8_t marker, const std::vector<uint8_t> &d) {
  o.push_back(0xFF);
  o.push_back(marker);
  o.push_back((uint8_t)((d.size() + 2) >> 8));
  o.push_back((uint8_t)(d.size() + 2));
  o.insert(o.end(), d.begin(), d.end());
}

void codes(const uint8_t bits[16], const uint8_t *vals, uint16_t *code, uint8_t *len) {
  uint32_t c = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    for (int i = 0; i < bits[l - 1]; i++, k++) {
      code[vals[k]] = (uint16_t)c;
      len[vals[k]] = (uint8_t)l;
      c++;
    }
    c <<= 1;
  }
}
}  // namespace

void jpeg_enc_qtables(int quality, uint8_t q[2][64]) {
  int s = quality < 1 ? 1 : quality > 100 ? 100 : quality;
  s = s < 50 ? 5000 / s : 200 - 2 * s;
  for (int i = 0; i < 64; i++) {
    const uint32_t a = ((uint32_t)kLumaQ[i] * (uint32_t)s + 50) / 100;
    const uint32_t b = ((uint32_t)kChromaQ[i] * (uint32_t)s + 50) / 100;
    q[0][i] = (uint8_t)(a < 1 ? 1 : a > 255 ? 255 : a);
    q[1][i] = (uint8_t)(b < 1 ? 1 : b > 255 ? 255 : b);
  }
}

std::vector<uint8_t> jpeg_enc_header(uint32_t w, uint32_t h, int ncomp, int quality) {
  std::vector<uint8_t> o = {0xFF, 0xD8};
  segment(o, 0xE0, {'J', 'F', 'I', 'F', 0, 1, 2, 0, 0, 1, 0, 1, 0, 0});
  std::vector<uint8_t> sof = {8, (uint8_t)(h >> 8), (uint8_t)h, (uint8_t)(w >> 8), (uint8_t)w, (uint8_t)ncomp};
  for (int c = 0; c < ncomp; c++) {
    sof.push_back((uint8_t)(c + 1));
    sof.push_back(0x11);
    sof.push_back((uint8_t)(c ? 1 : 0));
  }
  segment(o, 0xC0, sof);
  uint8_t q[2][64];
  jpeg_enc_qtables(quality, q);
  for (int t = 0; t < (ncomp == 1 ? 1 : 2); t++) {
    std::vector<uint8_t> d = {(uint8_t)t};
    for (int i = 0; i < 64; i++) d.push_back(q[t][kZigzag[i]]);
    segment(o, 0xDB, d);
  }
  const uint8_t *bits[4] = {kDcLumaBits, kAcLumaBits, kDcChromaBits, kAcChromaBits};
  const uint8_t *vals[4] = {kDcVals, kAcLumaVals, kDcVals, kAcChromaVals};
  const uint8_t cls[4] = {0x00, 0x10, 0x01, 0x11};
  for (int t = 0; t < (ncomp == 1 ? 2 : 4); t++) {
    std::vector<uint8_t> d = {cls[t]};
    int nv = 0;
    for (int i = 0; i < 16; i++) {
      d.push_back(bits[t][i]);
      nv += bits[t][i];
    }
    d.insert(d.end(), vals[t], vals[t] + nv);
    segment(o, 0xC4, d);
  }
  std::vector<uint8_t> sos = {(uint8_t)ncomp};
  for (int c = 0; c < ncomp; c++) {
    sos.push_back((uint8_t)(c + 1));
    sos.push_back(c ? 0x11 : 0x00);
  }
  sos.push_back(0);
  sos.push_back(63);
  sos.push_back(0);
  segment(o, 0xDA, sos);
  return o;
}

void jpeg_enc_tables(EncTables &t) {
  memset(&t, 0, sizeof(t));
  codes(kDcLumaBits, kDcVals, t.code[0], t.len[0]);
  codes(kAcLumaBits, kAcLumaVals, t.code[1], t.len[1]);
  codes(kDcChromaBits, kDcVals, t.code[2], t.len[2]);
  codes(kAcChromaBits, kAcChromaVals, t.code[3], t.len[3]);
}

uint64_t jpeg_enc_bound(uint32_t w, uint32_t h, uint32_t C) {
  const uint64_t ncomp = C <= 2 ? 1 : 3;
  const uint64_t blocks = (uint64_t)((w + 7) / 8) * ((h + 7) / 8) * ncomp;
  return 1024 + blocks * 420;  // a block codes to <= 1665 bits; stuffing at most doubles it
}

}  // namespace dg
