// dg_penc.hip — PNG re-encode of transformed images on the GPU
// (pre_encode_images with encode_format "png", image_processing.rs:396-413:
// image 0.25's PngEncoder, CompressionType::Fast, FilterType::Adaptive).
//
//   k_penc_filter  one wave per row: the five PNG filters (spec 9.2), the one
//                  with the smallest sum of |byte as i8| is kept (adaptive
//                  heuristic, PNG spec 12.8), filtered row -> the stream
//   k_penc_count   one thread per 1 KiB piece of the filtered stream: greedy
//                  run-length parse (DEFLATE matches at distance 1), bits of
//                  the piece under the fixed Huffman code, Adler-32 partials
//   k_enc_scan     (dg_enc.hip) exclusive scan of the piece bit lengths
//   k_penc_write   one thread per piece: the codes OR-ed LSB-first into the
//                  zeroed bit buffer at the piece's offset
//   k_penc_final   one workgroup per image: PNG signature + IHDR (host bytes),
//                  IDAT = zlib(78 01, one fixed-Huffman block, Adler-32),
//                  chunk CRC-32 (parallel slices combined with a GF(2)
//                  shift operator), IEND
//
// The byte stream is not the png crate's (fdeflate 0.3.7's "Fast" compressor
// is not vendored offline, so its exact output is unpinnable); what is pinned
// is the format: PIL and zlib read the file, CRCs and Adler-32 check, and the
// decoded pixels equal the encoder's input bit for bit.
#include <hip/hip_runtime.h>

#include "dg_types.h"
#include "kernels.h"

namespace dg {

// ------------------------------------------------------------ filter

__device__ __forceinline__ uint32_t paeth_pred(uint32_t a, uint32_t b, uint32_t c) {
  const int32_t p = (int32_t)a + (int32_t)b - (int32_t)c;
  const int32_t pa = abs(p - (int32_t)a), pb = abs(p - (int32_t)b), pc = abs(p - (int32_t)c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

__device__ __forceinline__ uint32_t filt_byte(uint32_t f, uint32_t x, uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t pr = f == 0 ? 0u : f == 1 ? a : f == 2 ? b : f == 3 ? (a + b) >> 1 : paeth_pred(a, b, c);
  return (x - pr) & 0xFFu;
}

__device__ __forceinline__ uint32_t abs_i8(uint32_t v) { return v < 128u ? v : 256u - v; }

// source row y of the encoder input (bpp bytes per pixel, rb bytes per row)
__device__ __forceinline__ const DG_GLOBAL uint8_t *penc_row(const EncDesc &e, uint32_t y) {
  return gp<const uint8_t>(e.src) + (size_t)y * e.src_stride;
}

__global__ __launch_bounds__(256) void k_penc_filter(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t y = it.item0 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (y >= e.h) return;
  const uint32_t bpp = e.C, rb = e.w * e.C;
  const DG_GLOBAL uint8_t *cur = penc_row(e, y), *up = y ? penc_row(e, y - 1) : nullptr;
  uint32_t sum[5] = {0, 0, 0, 0, 0};
  for (uint32_t x = lane; x < rb; x += 64) {
    const uint32_t v = cur[x], a = x >= bpp ? cur[x - bpp] : 0u, b = up ? up[x] : 0u,
                   c = (up && x >= bpp) ? up[x - bpp] : 0u;
#pragma unroll
    for (uint32_t f = 0; f < 5; f++) sum[f] += abs_i8(filt_byte(f, v, a, b, c));
  }
  uint32_t best = 0, bs = 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t f = 0; f < 5; f++) {
    uint32_t s = sum[f];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (s < bs) {  // ties keep the lower filter type
      bs = s;
      best = f;
    }
  }
  DG_GLOBAL uint8_t *dst = gp<uint8_t>(e.coef) + (size_t)y * (rb + 1);
  if (lane == 0) dst[0] = (uint8_t)best;
  for (uint32_t x = lane; x < rb; x += 64) {
    const uint32_t v = cur[x], a = x >= bpp ? cur[x - bpp] : 0u, b = up ? up[x] : 0u,
                   c = (up && x >= bpp) ? up[x - bpp] : 0u;
    dst[1 + x] = (uint8_t)filt_byte(best, v, a, b, c);
  }
}

// ------------------------------------------------------------ DEFLATE (fixed Huffman, RFC 1951 3.2.6)

constexpr uint32_t kPencPiece = 1024;  // filtered bytes per parse thread
constexpr uint32_t kAdlerMod = 65521;

// bit-reversed fixed code of a literal/length symbol: (code, length)
__device__ __forceinline__ void fixed_code(uint32_t sym, uint32_t &code, uint32_t &len) {
  uint32_t c;
  if (sym < 144) {
    c = 0x30u + sym;
    len = 8;
  } else if (sym < 256) {
    c = 0x190u + (sym - 144);
    len = 9;
  } else if (sym < 280) {
    c = sym - 256;
    len = 7;
  } else {
    c = 0xC0u + (sym - 280);
    len = 8;
  }
  code = __builtin_bitreverse32(c) >> (32 - len);  // Huffman codes go MSB first into an LSB-first stream
}

// length 3..258 -> symbol 257..285, extra bits and their value
__device__ __forceinline__ void len_code(uint32_t L, uint32_t &sym, uint32_t &eb, uint32_t &ev) {
  if (L == 258) {
    sym = 285;
    eb = 0;
    ev = 0;
    return;
  }
  if (L < 11) {
    sym = 254 + L;
    eb = 0;
    ev = 0;
    return;
  }
  // L - 3 = (4 + m) << e | r with e = extra bits: symbols 265.. in groups of 4
  const uint32_t d = L - 3;
  const uint32_t e = 31u - __builtin_clz(d) - 2u;  // d >= 8
  sym = 257 + 4 * (e + 1) + ((d >> e) - 4);
  eb = e;
  ev = d & ((1u << e) - 1u);
}

// Greedy parse of [p0, p1): a run of >= 3 bytes equal to the byte before is
// one match at distance 1 (length 3..258); everything else a literal.
template <class Emit>
__device__ __forceinline__ void penc_parse(const DG_GLOBAL uint8_t *s, uint32_t p0, uint32_t p1, Emit emit) {
  uint32_t i = p0;
  while (i < p1) {
    if (i > 0) {
      const uint32_t prev = s[i - 1];
      uint32_t k = 0;
      while (k < 258 && i + k < p1 && s[i + k] == prev) k++;
      if (k >= 3) {
        uint32_t sym, eb, ev, code, len;
        len_code(k, sym, eb, ev);
        fixed_code(sym, code, len);
        emit(code, len);
        if (eb) emit(ev, eb);
        emit(0u, 5u);  // distance code 0 (distance 1), 5 bits, no extra
        i += k;
        continue;
      }
    }
    uint32_t code, len;
    fixed_code(s[i], code, len);
    emit(code, len);
    i++;
  }
}

__global__ __launch_bounds__(256) void k_penc_count(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t pc = it.item0 + threadIdx.x;
  if (pc >= e.nblocks) return;
  const uint32_t N = e.h * (e.w * e.C + 1);
  const uint32_t p0 = pc * kPencPiece, p1 = min(p0 + kPencPiece, N);
  const DG_GLOBAL uint8_t *s = gp<const uint8_t>(e.coef);
  uint32_t bits = 0;
  penc_parse(s, p0, p1, [&](uint32_t, uint32_t n) { bits += n; });
  gp<uint32_t>(e.bits)[pc] = bits;
  // Adler-32 partials: S = sum of bytes, T = sum (L - j) * byte_j, both mod 65521
  uint64_t S = 0, T = 0;
  const uint32_t L = p1 - p0;
  for (uint32_t j = 0; j < L; j++) {
    const uint32_t v = s[p0 + j];
    S += v;
    T += (uint64_t)(L - j) * v;
  }
  DG_GLOBAL uint32_t *adl = gp<uint32_t>(e.aux) + 2 * (size_t)pc;
  adl[0] = (uint32_t)(S % kAdlerMod);
  adl[1] = (uint32_t)(T % kAdlerMod);
}

__global__ __launch_bounds__(256) void k_penc_write(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t pc = it.item0 + threadIdx.x;
  if (pc >= e.nblocks) return;
  const uint32_t N = e.h * (e.w * e.C + 1);
  const uint32_t p0 = pc * kPencPiece, p1 = min(p0 + kPencPiece, N);
  const DG_GLOBAL uint8_t *s = gp<const uint8_t>(e.coef);
  DG_GLOBAL uint32_t *w = gp<uint32_t>(e.words);
  // stream bit k = bit (k & 31) of word k >> 5 (little-endian words = the byte stream)
  uint32_t pos = 3u + gp<const uint32_t>(e.bits)[pc];  // after the 3-bit block header
  uint64_t acc = 0;
  uint32_t nacc = pos & 31u, wi = pos >> 5;
  auto emit = [&](uint32_t v, uint32_t n) {
    acc |= (uint64_t)v << nacc;
    nacc += n;
    if (nacc >= 32) {
      atomicOr((uint32_t *)&w[wi], (uint32_t)acc);
      acc >>= 32;
      nacc -= 32;
      wi++;
    }
  };
  penc_parse(s, p0, p1, emit);
  if (nacc) atomicOr((uint32_t *)&w[wi], (uint32_t)acc);
  if (pc == 0) atomicOr((uint32_t *)&w[0], 3u);  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
}

// ------------------------------------------------------------ container

// CRC-32 (PNG spec 5.5, reflected polynomial 0xEDB88320)
struct CrcSmem {
  uint32_t tab[256];
  uint32_t reg[1024];
  uint32_t mL[32], mLast[32];
};

// GF(2) operator: v -> the CRC register after feeding `bytes` zero bytes
__device__ uint32_t gf2_apply(const uint32_t *m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; i++, v >>= 1)
    if (v & 1u) r ^= m[i];
  return r;
}
__device__ void gf2_square(uint32_t *dst, const uint32_t *m) {
  for (int i = 0; i < 32; i++) dst[i] = gf2_apply(m, m[i]);
}
// m = operator for n zero bytes (n >= 0)
__device__ void crc_shift_op(uint32_t *m, uint64_t n) {
  uint32_t b[32], tmp[32];  // b: one zero bit, then squared to bytes
  b[0] = 0xEDB88320u;
  for (int i = 1; i < 32; i++) b[i] = 1u << (i - 1);
  for (int i = 0; i < 32; i++) m[i] = 1u << i;  // identity
  uint32_t sq[32];
  gf2_square(sq, b);  // 2 bits
  gf2_square(b, sq);  // 4 bits
  gf2_square(sq, b);  // 8 bits = one byte
  for (int i = 0; i < 32; i++) b[i] = sq[i];
  while (n) {
    if (n & 1) {
      for (int i = 0; i < 32; i++) tmp[i] = gf2_apply(b, m[i]);
      for (int i = 0; i < 32; i++) m[i] = tmp[i];
    }
    n >>= 1;
    if (n) {
      gf2_square(sq, b);
      for (int i = 0; i < 32; i++) b[i] = sq[i];
    }
  }
}

__device__ __forceinline__ void put_be32(DG_GLOBAL uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

__global__ __launch_bounds__(1024) void k_penc_final(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ CrcSmem sm;
  __shared__ uint32_t adler_s;
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  if (im.status) return;
  EncDesc &e = im.enc;
  const uint32_t t = threadIdx.x;
  const uint32_t N = e.h * (e.w * e.C + 1);
  const uint32_t dbits = 3u + e.total_bits + 7u;  // header, pieces, end-of-block (7 zero bits)
  const uint32_t dbytes = (dbits + 7) / 8;
  const uint32_t zlen = 2 + dbytes + 4;
  DG_GLOBAL uint8_t *out = gp<uint8_t>(e.out);
  const DG_GLOBAL uint8_t *hdr = gp<const uint8_t>(e.hdr);  // signature + IHDR chunk
  const uint32_t H0 = e.hdr_len;                             // 33
  // deflate bytes straight from the bit buffer
  const DG_GLOBAL uint8_t *db = gp<const uint8_t>(e.words);
  for (uint32_t i = t; i < dbytes; i += 1024) out[H0 + 10 + i] = db[i];
  for (uint32_t i = t; i < H0; i += 1024) out[i] = hdr[i];
  for (uint32_t i = t; i < 256; i += 1024) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    sm.tab[i] = c;
  }
  if (t == 0) {
    put_be32(out + H0, zlen);
    out[H0 + 4] = 'I';
    out[H0 + 5] = 'D';
    out[H0 + 6] = 'A';
    out[H0 + 7] = 'T';
    out[H0 + 8] = 0x78;  // zlib: deflate, 32 KiB window
    out[H0 + 9] = 0x01;  //       fastest level, FCHECK: 0x7801 % 31 == 0
    // Adler-32 of the filtered stream from the piece partials
    const DG_GLOBAL uint32_t *adl = gp<const uint32_t>(e.aux);
    uint64_t A = 1, B = N % kAdlerMod;
    for (uint32_t pc = 0; pc < e.nblocks; pc++) {
      const uint32_t p0 = pc * kPencPiece, p1 = min(p0 + kPencPiece, N);
      const uint64_t R = (uint64_t)(N - p1) % kAdlerMod;  // bytes after the piece
      A += adl[2 * pc];
      B += (uint64_t)adl[2 * pc] * R + adl[2 * pc + 1];
      A %= kAdlerMod;
      B %= kAdlerMod;
    }
    adler_s = (uint32_t)((B << 16) | A);
    put_be32(out + H0 + 10 + dbytes, adler_s);
  }
  __syncthreads();
  // CRC-32 over "IDAT" + zlib data: equal slices per thread, combined in order
  const uint32_t cb = H0 + 4, cn = 4 + zlen;  // first byte, length
  const uint32_t per = (cn + 1023) / 1024;
  const uint32_t s0 = min(t * per, cn), s1 = min(s0 + per, cn);
  uint32_t reg = 0;
  for (uint32_t i = s0; i < s1; i++) reg = sm.tab[(reg ^ out[cb + i]) & 0xFFu] ^ (reg >> 8);
  sm.reg[t] = reg;
  const uint32_t nsl = (cn + per - 1) / per;  // non-empty slices
  const uint32_t last = cn - (nsl - 1) * per;
  if (t == 0) crc_shift_op(sm.mL, per);
  if (t == 64) crc_shift_op(sm.mLast, last);
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < nsl; k++) acc = gf2_apply(k + 1 < nsl ? sm.mL : sm.mLast, acc) ^ sm.reg[k];
    const uint32_t crc = ~acc;
    DG_GLOBAL uint8_t *q = out + H0 + 10 + dbytes + 4;
    put_be32(q, crc);
    const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
    for (int i = 0; i < 12; i++) q[4 + i] = iend[i];
    e.enc_bytes = H0 + 10 + dbytes + 4 + 4 + 12;
  }
}

// ------------------------------------------------------------ launchers

void launch_penc_filter(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_penc_filter, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_penc_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_penc_count, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_penc_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_penc_write, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_penc_final(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_penc_final, dim3(nwg), dim3(1024), 0, st, imgs, list);
}

}  // namespace dg
