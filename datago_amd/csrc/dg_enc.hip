// dg_enc.hip — CDNA4 (gfx950) kernels of the JPEG re-encode step
// (pre_encode_images with encode_format "jpeg", reference
// image_processing.rs:374-395 -> image 0.25.9 JpegEncoder::new_with_quality).
//
//   k_enc_fdct   one thread per MCU: RGB -> YCbCr (f32, truncating), edge
//                replication, integer FDCT (jfdctint islow), quantisation
//                ((coef / 8) as f32 / q).round(); int16 zigzag blocks
//   k_enc_count  one thread per block: Huffman bit length (DC difference to
//                the previous block of the same component)
//   k_enc_scan   one workgroup per image: exclusive scan of the bit lengths
//   k_enc_write  one thread per block: codes OR-ed into the zeroed bit buffer
//                at the block's offset (only the words shared with the
//                neighbouring blocks ever see two writers)
//   k_enc_stuff  one workgroup per image: header copy, 0xFF -> 0xFF 0x00
//                stuffing with a block-wide scan, 1-bit padding, EOI
// oracle/jpeg_enc_oracle.c is the CPU restatement the tests compare against
// byte for byte.  All of it is integer/byte work except the colour
// conversion and the quantisation divide (f32, IEEE, no contraction).
#include <hip/hip_runtime.h>

#include "dg_types.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace dg {

__device__ __forceinline__ uint8_t sat_u8(float v) { return (uint8_t)(v <= 0.0f ? 0 : v >= 255.0f ? 255 : (int)v); }

constexpr int kCB = 13, kP1 = 2;
__device__ __forceinline__ void fdct8x8(int32_t *c) {
#pragma unroll
  for (int y = 0; y < 8; y++) {
    int32_t *s = c + y * 8;
    int32_t t0 = s[0] + s[7], t1 = s[1] + s[6], t2 = s[2] + s[5], t3 = s[3] + s[4];
    const int32_t t10 = t0 + t3, t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
    t0 = s[0] - s[7];
    t1 = s[1] - s[6];
    t2 = s[2] - s[5];
    t3 = s[3] - s[4];
    s[0] = (t10 + t11 - 8 * 128) << kP1;
    s[4] = (t10 - t11) << kP1;
    int32_t z1 = (t12 + t13) * 4433 + (1 << (kCB - kP1 - 1));
    s[2] = (z1 + t12 * 6270) >> (kCB - kP1);
    s[6] = (z1 - t13 * 15137) >> (kCB - kP1);
    int32_t u12 = t0 + t2, u13 = t1 + t3;
    z1 = (u12 + u13) * 9633 + (1 << (kCB - kP1 - 1));
    u12 = u12 * (-3196) + z1;
    u13 = u13 * (-16069) + z1;
    z1 = (t0 + t3) * (-7373);
    const int32_t v0 = t0 * 12299 + z1 + u12, v3 = t3 * 2446 + z1 + u13;
    z1 = (t1 + t2) * (-20995);
    const int32_t v1 = t1 * 25172 + z1 + u13, v2 = t2 * 16819 + z1 + u12;
    s[1] = v0 >> (kCB - kP1);
    s[3] = v1 >> (kCB - kP1);
    s[5] = v2 >> (kCB - kP1);
    s[7] = v3 >> (kCB - kP1);
  }
#pragma unroll
  for (int x = 0; x < 8; x++) {
    int32_t *s = c + x;
    int32_t t0 = s[0] + s[56], t1 = s[8] + s[48], t2 = s[16] + s[40], t3 = s[24] + s[32];
    const int32_t t10 = t0 + t3 + (1 << (kP1 - 1)), t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
    t0 = s[0] - s[56];
    t1 = s[8] - s[48];
    t2 = s[16] - s[40];
    t3 = s[24] - s[32];
    s[0] = (t10 + t11) >> kP1;
    s[32] = (t10 - t11) >> kP1;
    int32_t z1 = (t12 + t13) * 4433 + (1 << (kCB + kP1 - 1));
    s[16] = (z1 + t12 * 6270) >> (kCB + kP1);
    s[48] = (z1 - t13 * 15137) >> (kCB + kP1);
    int32_t u12 = t0 + t2, u13 = t1 + t3;
    z1 = (u12 + u13) * 9633 + (1 << (kCB + kP1 - 1));
    u12 = u12 * (-3196) + z1;
    u13 = u13 * (-16069) + z1;
    z1 = (t0 + t3) * (-7373);
    const int32_t v0 = t0 * 12299 + z1 + u12, v3 = t3 * 2446 + z1 + u13;
    z1 = (t1 + t2) * (-20995);
    const int32_t v1 = t1 * 25172 + z1 + u13, v2 = t2 * 16819 + z1 + u12;
    s[8] = v0 >> (kCB + kP1);
    s[24] = v1 >> (kCB + kP1);
    s[40] = v2 >> (kCB + kP1);
    s[56] = v3 >> (kCB + kP1);
  }
}

// One thread per MCU (8x8 pixels, all components).
__global__ __launch_bounds__(256) void k_enc_fdct(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t mcu = it.item0 + threadIdx.x;
  if (mcu >= e.nbx * e.nby) return;
  const uint32_t by = mcu / e.nbx, bx = mcu - by * e.nbx;
  const DG_GLOBAL uint8_t *src = gp<const uint8_t>(e.src);
  int32_t blk[3][64];
#pragma unroll
  for (int y = 0; y < 8; y++) {
    const uint32_t sy = min(by * 8 + y, e.h - 1);
#pragma unroll
    for (int x = 0; x < 8; x++) {
      const uint32_t sx = min(bx * 8 + x, e.w - 1);
      if (e.ncomp == 1) {
        uint32_t v;
        if (e.mode == 1) {  // GrayImage over a resized LA buffer: luma byte sy*w + sx of the LA bytes
          const uint32_t i = sy * e.w + sx, rb = 2 * e.w, r = i / rb;
          v = src[(size_t)r * e.src_stride + (i - r * rb)];
        } else {
          v = src[(size_t)sy * e.src_stride + (size_t)sx * e.C];
        }
        blk[0][y * 8 + x] = (int32_t)v;
      } else {
        const DG_GLOBAL uint8_t *p = src + (size_t)sy * e.src_stride + (size_t)sx * e.C;
        const float mx = 255.0f;
        const float r = (float)p[0], g = (float)p[1], b = (float)p[2];
        const float yy = 76.245f / mx * r + 149.685f / mx * g + 29.07f / mx * b;
        const float cb = -43.0185f / mx * r - 84.4815f / mx * g + 127.5f / mx * b + 128.0f;
        const float cr = 127.5f / mx * r - 106.7685f / mx * g - 20.7315f / mx * b + 128.0f;
        blk[0][y * 8 + x] = sat_u8(yy);
        blk[1][y * 8 + x] = sat_u8(cb);
        blk[2][y * 8 + x] = sat_u8(cr);
      }
    }
  }
  DG_GLOBAL int16_t *co = gp<int16_t>(e.coef) + (size_t)mcu * e.ncomp * 64;
#pragma unroll
  for (uint32_t c = 0; c < 3; c++) {
    if (c >= e.ncomp) break;
    fdct8x8(blk[c]);
#pragma unroll
    for (int k = 0; k < 64; k++) {
      constexpr uint8_t zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                  35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                  58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
      const uint32_t n = zz[k];
      const float v = (float)(blk[c][n] / 8) / (float)e.q[c ? 1 : 0][n];
      co[c * 64 + k] = (int16_t)roundf(v);
    }
  }
}

__device__ __forceinline__ uint32_t magnitude_bits(int32_t v) {
  const uint32_t a = (uint32_t)(v < 0 ? -v : v);
  return a ? 32u - (uint32_t)__clz(a) : 0u;
}

// Visit the Huffman codes of block b: emit(code, len) then emit(bits, n) per symbol.
template <class F>
__device__ __forceinline__ void enc_block(const EncDesc &e, const EncTables *T, uint32_t b, F emit) {
  const DG_GLOBAL int16_t *co = gp<const int16_t>(e.coef) + (size_t)b * 64;
  const uint32_t c = b % e.ncomp;
  const int32_t prev = b >= e.ncomp ? (int32_t)(gp<const int16_t>(e.coef)[(size_t)(b - e.ncomp) * 64]) : 0;
  const uint32_t t = c ? 2 : 0;
  const int32_t diff = (int32_t)co[0] - prev;
  uint32_t sz = magnitude_bits(diff);
  emit(T->code[t][sz], T->len[t][sz]);
  if (sz) emit(diff < 0 ? (uint32_t)(diff - 1) & ((1u << sz) - 1u) : (uint32_t)diff, sz);
  uint32_t run = 0;
  int32_t v63 = 0;
  for (uint32_t k = 1; k < 64; k++) {
    const int32_t v = co[k];
    if (k == 63) v63 = v;
    if (v == 0) {
      run++;
      continue;
    }
    while (run > 15) {
      emit(T->code[t + 1][0xF0], T->len[t + 1][0xF0]);
      run -= 16;
    }
    sz = magnitude_bits(v);
    const uint32_t sym = (run << 4) | sz;
    emit(T->code[t + 1][sym], T->len[t + 1][sym]);
    emit(v < 0 ? (uint32_t)(v - 1) & ((1u << sz) - 1u) : (uint32_t)v, sz);
    run = 0;
  }
  if (v63 == 0) emit(T->code[t + 1][0x00], T->len[t + 1][0x00]);
}

__global__ __launch_bounds__(256) void k_enc_count(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t b = it.item0 + threadIdx.x;
  if (b >= e.nblocks) return;
  const EncTables *T = (const EncTables *)(uintptr_t)e.tab;
  uint32_t n = 0;
  enc_block(e, T, b, [&](uint32_t, uint32_t len) { n += len; });
  gp<uint32_t>(e.bits)[b] = n;
}

// One 1024-thread workgroup per image: bits[] -> exclusive offsets, total.
__global__ __launch_bounds__(1024) void k_enc_scan(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ uint32_t part[1024];
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  if (im.status) return;
  EncDesc &e = im.enc;
  DG_GLOBAL uint32_t *bits = gp<uint32_t>(e.bits);
  const uint32_t n = e.nblocks, t = threadIdx.x;
  const uint32_t per = (n + 1023) / 1024, b0 = min(t * per, n), b1 = min(b0 + per, n);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; b++) s += bits[b];
  part[t] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (uint32_t b = b0; b < b1; b++) {
    const uint32_t x = bits[b];
    bits[b] = run;
    run += x;
  }
  if (t == 1023) e.total_bits = part[1023];
}

__global__ __launch_bounds__(256) void k_enc_write(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const EncDesc &e = im.enc;
  const uint32_t b = it.item0 + threadIdx.x;
  if (b >= e.nblocks) return;
  const EncTables *T = (const EncTables *)(uintptr_t)e.tab;
  DG_GLOBAL uint32_t *w = gp<uint32_t>(e.words);
  const uint32_t p0 = gp<const uint32_t>(e.bits)[b];
  uint32_t wi = p0 >> 5, nb = p0 & 31u;
  uint64_t acc = 0;  // stream bits, MSB first, from word wi
  enc_block(e, T, b, [&](uint32_t v, uint32_t len) {
    acc |= (uint64_t)v << (64 - nb - len);
    nb += len;
    if (nb >= 32) {
      atomicOr((uint32_t *)&w[wi], __builtin_bswap32((uint32_t)(acc >> 32)));
      acc <<= 32;
      nb -= 32;
      wi++;
    }
  });
  if (nb) atomicOr((uint32_t *)&w[wi], __builtin_bswap32((uint32_t)(acc >> 32)));
}

// One 1024-thread workgroup per image: header, stuffed scan, padding, EOI.
__global__ __launch_bounds__(1024) void k_enc_stuff(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ uint32_t part[1024];
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  if (im.status) return;
  EncDesc &e = im.enc;
  if (e.png) return;  // PNG re-encode: k_penc_final
  const uint32_t t = threadIdx.x;
  DG_GLOBAL uint8_t *out = gp<uint8_t>(e.out);
  const DG_GLOBAL uint8_t *hdr = gp<const uint8_t>(e.hdr);
  for (uint32_t i = t; i < e.hdr_len; i += 1024) out[i] = hdr[i];
  const uint32_t tb = e.total_bits, nbytes = (tb + 7) / 8, rem = tb & 7u;
  const DG_GLOBAL uint8_t *sb = gp<const uint8_t>(e.words);
  uint32_t base = e.hdr_len;
  for (uint32_t b0 = 0; b0 < nbytes; b0 += 4096) {  // 4 bytes per thread per round
    uint8_t v[4];
    uint32_t ff = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t i = b0 + 4 * t + k;
      uint8_t x = i < nbytes ? sb[i] : 0;
      if (rem && i == nbytes - 1) x |= (uint8_t)((1u << (8 - rem)) - 1u);  // pad with 1-bits
      v[k] = x;
      ff += (i < nbytes && x == 0xFF) ? 1u : 0u;
    }
    const uint32_t mine = (b0 + 4 * t < nbytes ? min(4u, nbytes - (b0 + 4 * t)) : 0u) + ff;
    part[t] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint32_t x = t >= o ? part[t - o] : 0u;
      __syncthreads();
      part[t] += x;
      __syncthreads();
    }
    uint32_t pos = base + part[t] - mine;
    const uint32_t total = part[1023];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t i = b0 + 4 * t + k;
      if (i < nbytes) {
        out[pos++] = v[k];
        if (v[k] == 0xFF) out[pos++] = 0;
      }
    }
    base += total;
    __syncthreads();
  }
  if (t == 0) {
    out[base] = 0xFF;
    out[base + 1] = 0xD9;
    e.enc_bytes = base + 2;
  }
}

// ------------------------------------------------------------ launchers

void launch_enc_fdct(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_enc_fdct, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_enc_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_enc_count, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_enc_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_enc_scan, dim3(nwg), dim3(1024), 0, st, imgs, list);
}
void launch_enc_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_enc_write, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_enc_stuff(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_enc_stuff, dim3(nwg), dim3(1024), 0, st, imgs, list);
}

}  // namespace dg
