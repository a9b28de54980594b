// kernels.hip — CDNA4 (gfx950) kernels of the decode + bucket-resize stage.
//
// Pipeline for one batch (all images at once, one HIP stream):
//   k_huff_sync   entropy decode, intra-workgroup self-synchronisation
//   k_huff_fix    cross-workgroup boundary repair (usually a no-op)
//   k_huff_scan   per-image segmented prefix of block counts / DC predictors
//   k_huff_write  final decode writing int16 zigzag coefficient blocks
//   k_coeffs      Lanczos3 i16 coefficient tables (fast_image_resize semantics)
//   k_idct        dequant + ISLOW IDCT -> component planes
//   k_color       fancy upsampling + YCbCr->RGB -> interleaved image
//   k_resize_hb   H passes in row bands (first pass of a colour image fused
//                 with upsampling + colour conversion); k_resize_h for
//                 segments wider than LDS
//   k_resize_v    V passes (R1.V, R2.V)
//   k_copy        exact-size images / gray->RGB expansion
// Everything is integer or byte work, so nothing here is MFMA-shaped; the
// design points are wave64 occupancy for the latency-bound entropy decoder,
// LDS-resident Huffman tables and coefficient blocks, coalesced row stores.
#include <hip/hip_runtime.h>

#include "dg_entropy.h"
#include "dg_pixel.h"
#include "dg_plane.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace dg {

// ------------------------------------------------------------------ helpers

__device__ __forceinline__ void load_tables(HuffTable *tabs, const HuffTable *pool, const ImageDesc &im) {
  const int words = (int)(sizeof(HuffTable) / 4);
  const int ns = im.nslots;
  for (int i = threadIdx.x; i < ns * words; i += blockDim.x) {
    int s = i / words, w = i - s * words;
    ((uint32_t *)&tabs[s])[w] = ((const uint32_t *)&pool[im.hslot[s]])[w];
  }
}

// ------------------------------------------------------------ destuffing
// Raw scan -> destuffed stream + RST marker positions, in three passes over
// 4 KiB raw chunks (count / per-image scan / write).  Each thread owns 16 raw
// bytes, read with six aligned dword loads that also cover its neighbours;
// chunks of 16 with no 0xFF byte (all but a few percent of them) are kept
// whole without per-byte work.  The write pass stages the chunk's kept bytes
// in LDS and stores them with aligned dwords.

struct Destuff16 {
  uint32_t kept, mks;  // kept bytes, RST markers among the 16
  uint32_t km, mm;     // per-byte keep / marker masks
  uint32_t r[4];       // the 16 raw bytes, little-endian
};

__device__ __forceinline__ bool has_ff(uint32_t x) {
  const uint32_t v = ~x;
  return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u;
}

__device__ __forceinline__ Destuff16 destuff16(const DG_GLOBAL uint8_t *raw, uint32_t n, uint32_t i0) {
  Destuff16 d;
  d.kept = d.mks = d.km = d.mm = 0;
  d.r[0] = d.r[1] = d.r[2] = d.r[3] = 0;
  if (i0 >= n) return d;
  if (i0 >= 4 && i0 + 24 <= n) {
    // bytes [i0 - 1, i0 + 17) from the aligned 24-byte window at A (inside the scan)
    const uintptr_t base = (uintptr_t)(raw + i0 - 1);
    const DG_GLOBAL uint32_t *w4 = (const DG_GLOBAL uint32_t *)(base & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(base & 3);
    uint32_t w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = w4[k];
    // window dwords starting at byte sh (prev = byte 0 of W0) and sh + 1 (the 16 raw bytes)
    uint32_t W[5];
#pragma unroll
    for (int m = 0; m < 5; m++) W[m] = __builtin_amdgcn_alignbyte(w[m + 1], w[m], sh);
    uint32_t R[4];
#pragma unroll
    for (int m = 0; m < 4; m++) R[m] = (W[m] >> 8) | (W[m + 1] << 24);
    const uint32_t prev = W[0] & 0xFFu;
    const uint32_t next = W[4] >> 8 & 0xFFu;  // byte i0 + 16
#pragma unroll
    for (int m = 0; m < 4; m++) d.r[m] = R[m];
    if (prev != 0xFFu && !has_ff(R[0]) && !has_ff(R[1]) && !has_ff(R[2]) && !has_ff(R[3])) {
      d.kept = 16;
      d.km = 0xFFFFu;
      return d;
    }
    uint32_t p = prev;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
      const uint32_t cur = (R[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const uint32_t nx = j < 15 ? (R[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xFFu : next;
      uint32_t mk;
      const uint32_t k = destuff_keep(p, cur, nx, false, &mk);
      d.km |= k << j;
      d.mm |= mk << j;
      d.kept += k;
      d.mks += mk;
      p = cur;
    }
    return d;
  }
  // scan head / tail: byte loads
  uint32_t prev = i0 ? raw[i0 - 1] : 0u;
  uint32_t cur = raw[i0];
  for (uint32_t j = 0; j < 16; j++) {
    const uint32_t i = i0 + j;
    if (i >= n) break;
    const uint32_t next = i + 1 < n ? raw[i + 1] : 0xD9u;
    d.r[j >> 2] |= cur << (8 * (j & 3));
    uint32_t mk;
    const uint32_t k = destuff_keep(prev, cur, next, i == 0, &mk);
    d.km |= k << j;
    d.mm |= mk << j;
    d.kept += k;
    d.mks += mk;
    prev = cur;
    cur = next;
  }
  return d;
}

__global__ __launch_bounds__(256) void k_destuff_count(const ImageDesc *__restrict__ imgs,
                                                       const WgItem *__restrict__ list) {
  __shared__ uint32_t rk[256], rm[256];
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const int t = threadIdx.x;
  const Destuff16 d = destuff16(gp<const uint8_t>(im.scan), im.scan_len, it.item0 * kDestuffChunk + t * 16);
  rk[t] = d.kept;
  rm[t] = d.mks;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) {
      rk[t] += rk[t + off];
      rm[t] += rm[t + off];
    }
    __syncthreads();
  }
  if (t == 0) {
    DG_GLOBAL uint32_t *ch = gp<uint32_t>(im.chunk) + it.item0 * 4;
    ch[0] = rk[0];
    ch[1] = rm[0];
  }
}

__global__ __launch_bounds__(256) void k_destuff_scan(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ uint32_t sk[256], sm[256];
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  const int t = threadIdx.x;
  DG_GLOBAL uint32_t *ch = gp<uint32_t>(im.chunk);
  uint32_t ck = 0, cm = 0;
  for (uint32_t c0 = 0; c0 < im.nchunk; c0 += 256) {
    uint32_t c = c0 + t;
    uint32_t k = c < im.nchunk ? ch[c * 4] : 0u, m = c < im.nchunk ? ch[c * 4 + 1] : 0u;
    sk[t] = k;
    sm[t] = m;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      uint32_t a = t >= off ? sk[t - off] : 0u, b = t >= off ? sm[t - off] : 0u;
      __syncthreads();
      sk[t] += a;
      sm[t] += b;
      __syncthreads();
    }
    if (c < im.nchunk) {
      ch[c * 4 + 2] = ck + sk[t] - k;
      ch[c * 4 + 3] = cm + sm[t] - m;
    }
    ck += sk[255];
    cm += sm[255];
    __syncthreads();
  }
  if (t == 0) {
    im.ds_bits = ck * 8;
    im.nmk = cm < im.mk_cap ? cm : im.mk_cap;
  }
  // zero padding (64 bytes) for the bit-window reader, in the interleaved layout
  DG_GLOBAL uint8_t *ds = gp<uint8_t>(im.ds);
  if (t < 64) {
    const uint32_t q = ck + t;
    ds[(size_t)ds_word_index(q >> 2, im.ds_lsw) * 4 + (q & 3)] = 0;
  }
}

__global__ __launch_bounds__(256) void k_destuff_write(const ImageDesc *__restrict__ imgs,
                                                       const WgItem *__restrict__ list) {
  __shared__ uint32_t sk[256], sm[256];
  __shared__ uint8_t buf[kDestuffChunk];
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const int t = threadIdx.x;
  const Destuff16 d = destuff16(gp<const uint8_t>(im.scan), im.scan_len, it.item0 * kDestuffChunk + t * 16);
  sk[t] = d.kept;
  sm[t] = d.mks;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t a = t >= off ? sk[t - off] : 0u, b = t >= off ? sm[t - off] : 0u;
    __syncthreads();
    sk[t] += a;
    sm[t] += b;
    __syncthreads();
  }
  const DG_GLOBAL uint32_t *ch = gp<const uint32_t>(im.chunk) + it.item0 * 4;
  const uint32_t O = ch[2];           // chunk's first output byte
  uint32_t o = sk[t] - d.kept;        // this thread's first byte within the chunk
  const uint32_t total = sk[255];
  if (d.km == 0xFFFFu) {
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) buf[o + j] = (uint8_t)(d.r[j >> 2] >> (8 * (j & 3)));
  } else {
    uint32_t mo = ch[3] + sm[t] - d.mks;
    DG_GLOBAL uint32_t *mk = gp<uint32_t>(im.mk);
    for (uint32_t j = 0; j < 16; j++) {
      if ((d.mm >> j) & 1u) {
        if (mo < im.mk_cap) mk[mo] = (O + o) * 8;
        mo++;
      }
      if ((d.km >> j) & 1u) buf[o++] = (uint8_t)(d.r[j >> 2] >> (8 * (j & 3)));
    }
  }
  __syncthreads();
  // buf[0, total) -> logical bytes [O, O + total) of the interleaved stream:
  // partial words at both ends byte by byte, whole words as dword stores
  DG_GLOBAL uint8_t *ds = gp<uint8_t>(im.ds);
  DG_GLOBAL uint32_t *ds4 = (DG_GLOBAL uint32_t *)ds;
  const uint32_t lsw = im.ds_lsw;
  const uint32_t mis = (4u - (O & 3u)) & 3u;  // bytes to the next word boundary
  const uint32_t head = mis < total ? mis : total;
  const uint32_t nd = (total - head) >> 2;
  if ((uint32_t)t < head) {
    const uint32_t q = O + t;
    ds[(size_t)ds_word_index(q >> 2, lsw) * 4 + (q & 3)] = buf[t];
  }
  const uint32_t w0 = (O + head) >> 2;  // first whole logical word
  for (uint32_t q = t; q < nd; q += 256) {
    const uint32_t b0 = head + 4 * q;
    ds4[ds_word_index(w0 + q, lsw)] = (uint32_t)buf[b0] | ((uint32_t)buf[b0 + 1] << 8) |
                                      ((uint32_t)buf[b0 + 2] << 16) | ((uint32_t)buf[b0 + 3] << 24);
  }
  const uint32_t tail0 = head + 4 * nd;
  if ((uint32_t)t < total - tail0) {
    const uint32_t q = O + tail0 + t;
    ds[(size_t)ds_word_index(q >> 2, lsw) * 4 + (q & 3)] = buf[tail0 + t];
  }
}

// Destuff in one pass (option "destuff_one"): count, prefix and write of a
// chunk in one workgroup, instead of k_destuff_count + k_destuff_scan +
// k_destuff_write (three launches, the raw scan read twice).  A chunk's
// output offset is the sum of its image's earlier chunks' kept bytes, found
// by decoupled look-back: each chunk publishes its own counts as soon as it
// has them (state word: bit 62 aggregate ready, bit 63 inclusive prefix
// ready, markers in bits 32..61, kept bytes in 0..31), then walks back over
// its predecessors' words, adding aggregates until it meets an inclusive
// prefix, and publishes its own inclusive prefix.  Chunks are taken in list
// order from a batch ticket (state[0]), so every predecessor was taken by a
// workgroup that is running or done: each wait ends.  A wait that does not
// end within ~1 s (a hardware or launch anomaly, never a property of the
// data) marks the image DG_ERR_UNSUPPORTED instead of hanging.  Wave 0 runs
// the look-back, 64 predecessors per round (one per lane), with wave-uniform
// control flow around the polling loop (see uf_wait in dg_png.hip).  A first
// version walked back one chunk per load (one L2 round trip each) and took
// 9.9 ms per batch instead of 0.44.  The state words carry their values
// with the flags, so they need atomicity and agent-scope coherence but no
// ordering of other memory: relaxed atomics.  Release/acquire at agent
// scope write back / invalidate the XCD's L2 on every publish and poll
// (MI355X's L2s are per XCD), and took 6.6 ms per batch even with the
// 64-wide look-back.
constexpr uint64_t kDsAgg = 1ull << 62, kDsIncl = 1ull << 63;

__global__ __launch_bounds__(256) void k_destuff_one(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                                     uint64_t *__restrict__ state) {
  __shared__ uint32_t sk[256], sm[256];
  __shared__ uint8_t buf[kDestuffChunk];
  __shared__ uint32_t s_item, s_ok, s_ek, s_em;
  const int t = threadIdx.x;
  if (t == 0) s_item = atomicAdd((uint32_t *)state, 1u);
  __syncthreads();
  const WgItem it = list[s_item];
  ImageDesc &im = imgs[it.image];
  const uint32_t c = it.item0;
  const Destuff16 d = destuff16(gp<const uint8_t>(im.scan), im.scan_len, c * kDestuffChunk + t * 16);
  sk[t] = d.kept;
  sm[t] = d.mks;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t a = t >= off ? sk[t - off] : 0u, b = t >= off ? sm[t - off] : 0u;
    __syncthreads();
    sk[t] += a;
    sm[t] += b;
    __syncthreads();
  }
  const uint32_t total = sk[255], mtotal = sm[255];
  uint64_t *cs = state + 1 + im.ds_state0;  // this image's chunk words
  if (t < 64) {  // wave 0
    const uint64_t own = ((uint64_t)(mtotal & 0x3FFFFFFFu) << 32) | total;
    uint32_t ek = 0, em = 0, ok = 1;
    if (c == 0) {
      __hip_atomic_store(cs, own | kDsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(cs + c, own | kDsAgg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // Look back 64 predecessors at a time, one per lane (lane l: chunk
      // base - 1 - l): the nearest inclusive prefix ends the walk, every
      // chunk between it and this one must have published its aggregate (a
      // window with a gap before its first inclusive word is read again).
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const uint32_t lane = t;
      uint32_t base = c;  // chunks [.., base) still to add
      for (;;) {
        const int32_t j = (int32_t)base - 1 - (int32_t)lane;
        const uint64_t v = j >= 0 ? __hip_atomic_load(cs + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kDsIncl;
        const uint64_t incl = __ballot((v & kDsIncl) != 0), none = __ballot((v & (kDsAgg | kDsIncl)) == 0);
        const uint32_t stop = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;  // first lane with a prefix
        const uint64_t before = stop >= 64 ? ~0ull : ((2ull << stop) - 1ull);  // lanes 0..stop
        if ((none & before) == 0) {  // lanes 0..stop all published: take them
          const bool take = lane <= stop && j >= 0;
          uint32_t vk = take ? (uint32_t)v : 0u, vm = take ? (uint32_t)(v >> 32) & 0x3FFFFFFFu : 0u;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            vk += __shfl_xor(vk, o);
            vm += __shfl_xor(vm, o);
          }
          ek += vk;
          em += vm;
          if (stop < 64) break;
          base -= 64;  // all 64 were aggregates: the next window
          continue;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // ~1 s at 100 MHz
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const uint64_t incl = ((uint64_t)((em + mtotal) & 0x3FFFFFFFu) << 32) | (uint64_t)(ek + total);
      __hip_atomic_store(cs + c, incl | kDsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) {
      s_ek = ek;
      s_em = em;
      s_ok = ok;
    }
  }
  __syncthreads();
  if (!s_ok) {
    if (t == 0) atomicCAS((int *)&im.status, 0, 1);  // DG_ERR_UNSUPPORTED (an earlier CORRUPT stays)
    return;  // uniform
  }
  const uint32_t O = s_ek;        // chunk's first output byte
  uint32_t o = sk[t] - d.kept;    // this thread's first byte within the chunk
  if (d.km == 0xFFFFu) {
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) buf[o + j] = (uint8_t)(d.r[j >> 2] >> (8 * (j & 3)));
  } else {
    uint32_t mo = s_em + sm[t] - d.mks;
    DG_GLOBAL uint32_t *mk = gp<uint32_t>(im.mk);
    for (uint32_t j = 0; j < 16; j++) {
      if ((d.mm >> j) & 1u) {
        if (mo < im.mk_cap) mk[mo] = (O + o) * 8;
        mo++;
      }
      if ((d.km >> j) & 1u) buf[o++] = (uint8_t)(d.r[j >> 2] >> (8 * (j & 3)));
    }
  }
  __syncthreads();
  DG_GLOBAL uint8_t *ds = gp<uint8_t>(im.ds);
  DG_GLOBAL uint32_t *ds4 = (DG_GLOBAL uint32_t *)ds;
  const uint32_t lsw = im.ds_lsw;
  const uint32_t mis = (4u - (O & 3u)) & 3u;
  const uint32_t head = mis < total ? mis : total;
  const uint32_t nd = (total - head) >> 2;
  if ((uint32_t)t < head) {
    const uint32_t q = O + t;
    ds[(size_t)ds_word_index(q >> 2, lsw) * 4 + (q & 3)] = buf[t];
  }
  const uint32_t w0 = (O + head) >> 2;
  for (uint32_t q = t; q < nd; q += 256) {
    const uint32_t b0 = head + 4 * q;
    ds4[ds_word_index(w0 + q, lsw)] = (uint32_t)buf[b0] | ((uint32_t)buf[b0 + 1] << 8) |
                                      ((uint32_t)buf[b0 + 2] << 16) | ((uint32_t)buf[b0 + 3] << 24);
  }
  const uint32_t tail0 = head + 4 * nd;
  if ((uint32_t)t < total - tail0) {
    const uint32_t q = O + tail0 + t;
    ds[(size_t)ds_word_index(q >> 2, lsw) * 4 + (q & 3)] = buf[tail0 + t];
  }
  if (c + 1 == im.nchunk) {  // the image's last chunk: stream length, marker count, zero padding
    const uint32_t ck = O + total, cm = s_em + mtotal;
    if (t == 0) {
      im.ds_bits = ck * 8;
      im.nmk = cm < im.mk_cap ? cm : im.mk_cap;
    }
    if (t < 64) {
      const uint32_t q = ck + t;
      ds[(size_t)ds_word_index(q >> 2, lsw) * 4 + (q & 3)] = 0;
    }
  }
}

// ------------------------------------------------------------ entropy decode

// debug: {start, end} of workgroup `rec` in s_memrealtime ticks (100 MHz)
__device__ __forceinline__ uint64_t wg_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void wg_time_store(const BatchFlags *flags, uint32_t rec, uint64_t t0) {
  if (flags->wgtime && threadIdx.x == 0) {
    DG_GLOBAL uint64_t *p = gp<uint64_t>(flags->wgtime) + 2 * (size_t)rec;
    p[0] = t0;
    p[1] = wg_clock();
  }
}

// Workgroup layout for sync/fix: 255 useful subsequences per workgroup.
// Thread 0 is a lead-in: it decodes the previous workgroup's last subsequence
// from a guessed state (writing nothing) so that thread 1 usually starts in
// step with the true decode and k_huff_fix finds nothing to repair.
constexpr uint32_t kUseful = kSubPerWg - 1;

__device__ __forceinline__ void store_sub(SubState &o, uint32_t in, uint32_t out, const RangeAcc &a,
                                          const StageCtx *stg = nullptr) {
  o.in = in;
  o.out = out;
  o.m = a.m;
  o.n = a.n;
  o.dc[0] = a.dc[0];
  o.dc[1] = a.dc[1];
  o.dc[2] = a.dc[2];
  if (stg && stg->on) {
    o.nstart = stg->started;
    o.nent = stg->n;
  }
}

// BatchFlags::prio (option "entropy_prio") as the wave's issue priority
__device__ __forceinline__ void entropy_setprio(const BatchFlags *flags) {
  const uint32_t p = __builtin_amdgcn_readfirstlane(flags->prio);
  if (p == 1) __builtin_amdgcn_s_setprio(1);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 3) __builtin_amdgcn_s_setprio(3);
}

template <bool STAGE>
__global__ __launch_bounds__(256) void k_huff_sync(const ImageDesc *__restrict__ imgs,
                                                   const WgItem *__restrict__ list,
                                                   const HuffTable *__restrict__ pool,
                                                   SubState *__restrict__ subs, Ckpt *__restrict__ ckpt,
                                                   BatchFlags *flags, uint32_t multi) {
  extern __shared__ __attribute__((aligned(16))) uint8_t huff_dyn[];  // im.nslots tables (launch: batch max)
  HuffTable *tabs = (HuffTable *)huff_dyn;
  __shared__ uint32_t ex[kSubPerWg], ins[kSubPerWg];
  const uint64_t t_start = wg_clock();
  entropy_setprio(flags);
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  load_tables(tabs, pool, im);
  // multi-symbol lookups of the image's distinct AC tables (after its tables;
  // the launch sizes the area for the batch's most), built from the LDS tables
  uint16_t *mt = (uint16_t *)(huff_dyn + (size_t)im.nslots * sizeof(HuffTable));
  uint32_t acm = 0xFFu, nac = 0, acs[kMultiLuts] = {0, 0, 0};
  for (uint32_t c = 0; c < im.ncomp && c < 4; c++) {
    const uint32_t sl = (im.slotmap >> ((2 * c + 1) * 4)) & 15u;
    uint32_t a = 3;
    for (uint32_t q = 0; q < nac; q++)
      if (acs[q] == sl) a = q;
    if (a == 3 && nac < kMultiLuts) {
      acs[nac] = sl;
      a = nac++;
    }
    acm = (acm & ~(3u << (2 * c))) | (a << (2 * c));
  }
  __syncthreads();
  if (multi & 1u) {
    for (uint32_t i = threadIdx.x; i < (nac << kMultiBits); i += blockDim.x) {
      const uint32_t q = i >> kMultiBits;
      const uint32_t sl = q == 0 ? acs[0] : q == 1 ? acs[1] : acs[2];
      mt[i] = (uint16_t)multi_entry(tabs[sl], i & ((1u << kMultiBits) - 1u));
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  const uint32_t s0 = it.item0;                  // first useful subsequence
  const int64_t si = (int64_t)s0 + t - 1;        // this thread's subsequence (t = 0: lead-in)
  const bool active = si >= 0 && si < (int64_t)im.nsub;
  const bool head = (t == 0) || (s0 == 0 && t == 1);
  const uint32_t s = active ? (uint32_t)si : 0u;
  const uint32_t nck = num_ckpt(im.sub_bits);
  // decode-once: record the coefficients (no checkpoint merging: a re-decode
  // must stage its whole range); thread 0's lead-in range belongs to the
  // previous workgroup and is not staged
  const bool stage = STAGE && im.stage != 0;
  DG_GLOBAL Ckpt *ck =
      (!stage && t > 0 && active && nck && im.ckpt) ? (DG_GLOBAL Ckpt *)ckpt + im.ckpt_base + (size_t)s * nck
                                                     : nullptr;
  StageCtx sc;
  sc.on = stage && t > 0 && active;
  sc.base = sc.on ? stage_range(im.stage, im.stage_cap, s) : nullptr;
  StageCtx *stg = STAGE ? &sc : nullptr;
  const DG_GLOBAL uint8_t *scan = gp<const uint8_t>(im.ds);
  const DG_GLOBAL uint32_t *mkp = gp<const uint32_t>(im.mk);
  RangeAcc acc = {0, 0, 0, {0, 0, 0}};
  // entry state: exact for s == 0, otherwise the lead-in decode's guess
  const bool pair = (multi & 2u) != 0;
  uint32_t in = active ? lead_in(im, tabs, scan, mkp, s, im.lead_bits, (multi & 1u) ? mt : nullptr, acm, pair)
                       : pack_state(0, 0, 0);
  if (active)
    decode_range<false>(im, tabs, scan, mkp, s, in, acc, nullptr, ck, false, 0, stg, (multi & 1u) ? mt : nullptr, acm,
                        pair);
  ex[t] = active ? acc.out : 0u;
  ins[t] = in;
  __syncthreads();
  uint32_t iters = 0;
  for (;;) {
    bool redo = active && !head && ins[t] != ex[t - 1];
    uint32_t pin = redo ? ex[t - 1] : 0u;
    __syncthreads();
    if (redo) {
      decode_range<false>(im, tabs, scan, mkp, s, pin, acc, nullptr, ck, true, ex[t], stg, (multi & 1u) ? mt : nullptr,
                          acm, pair);
      ex[t] = acc.out;
      ins[t] = pin;
    }
    iters++;
    if (!__syncthreads_or(redo)) break;
  }
  if (active && t > 0) store_sub(subs[im.sub_base + s], ins[t], ex[t], acc, stg);
  if (t == 0) atomicMax(&flags->sync_iters_max, iters);
  wg_time_store(flags, blockIdx.x, t_start);
}

// k_huff_sync with two chains per lane (option "sync2"):
// the same 256 slots per workgroup (slot 0 the lead-in slot, 255 useful
// subsequences, so k_huff_fix, k_huff_scan and the work lists are unchanged)
// on 128 threads, thread t owning slots t and t + 128.  Each thread runs both
// slots' lead-in + range decodes in lockstep (SyncChain, dg_entropy.h): two
// independent lookup chains per lane instead of one.  The verification loop
// is k_huff_sync's over the 256 slots; its rare re-decodes run per slot.
__global__ __launch_bounds__(128) void k_huff_sync2(const ImageDesc *__restrict__ imgs,
                                                    const WgItem *__restrict__ list,
                                                    const HuffTable *__restrict__ pool,
                                                    SubState *__restrict__ subs, Ckpt *__restrict__ ckpt,
                                                    BatchFlags *flags, uint32_t multi) {
  extern __shared__ __attribute__((aligned(16))) uint8_t huff_dyn[];
  HuffTable *tabs = (HuffTable *)huff_dyn;
  __shared__ uint32_t ex[kSubPerWg], ins[kSubPerWg];
  const uint64_t t_start = wg_clock();
  entropy_setprio(flags);
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  load_tables(tabs, pool, im);
  uint16_t *mt = (uint16_t *)(huff_dyn + (size_t)im.nslots * sizeof(HuffTable));
  uint32_t acm = 0xFFu, nac = 0, acs[kMultiLuts] = {0, 0, 0};
  for (uint32_t c = 0; c < im.ncomp && c < 4; c++) {
    const uint32_t sl = (im.slotmap >> ((2 * c + 1) * 4)) & 15u;
    uint32_t a = 3;
    for (uint32_t q = 0; q < nac; q++)
      if (acs[q] == sl) a = q;
    if (a == 3 && nac < kMultiLuts) {
      acs[nac] = sl;
      a = nac++;
    }
    acm = (acm & ~(3u << (2 * c))) | (a << (2 * c));
  }
  __syncthreads();
  if (multi & 1u) {
    for (uint32_t i = threadIdx.x; i < (nac << kMultiBits); i += blockDim.x) {
      const uint32_t q = i >> kMultiBits;
      const uint32_t sl = q == 0 ? acs[0] : q == 1 ? acs[1] : acs[2];
      mt[i] = (uint16_t)multi_entry(tabs[sl], i & ((1u << kMultiBits) - 1u));
    }
  }
  __syncthreads();
  const uint16_t *mtp = (multi & 1u) ? mt : nullptr;
  const int t = threadIdx.x;
  const uint32_t s0 = it.item0;  // first useful subsequence
  const uint32_t nck = num_ckpt(im.sub_bits);
  const DG_GLOBAL uint8_t *scan = gp<const uint8_t>(im.ds);
  const DG_GLOBAL uint32_t *mkp = gp<const uint32_t>(im.mk);
  bool active[2], head[2];
  uint32_t sv[2];
  DG_GLOBAL Ckpt *ckv[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int q = t + 128 * h;                      // slot
    const int64_t si = (int64_t)s0 + q - 1;         // its subsequence (q = 0: lead-in)
    active[h] = si >= 0 && si < (int64_t)im.nsub;
    head[h] = (q == 0) || (s0 == 0 && q == 1);
    sv[h] = active[h] ? (uint32_t)si : 0u;
    ckv[h] = (q > 0 && active[h] && nck && im.ckpt) ? (DG_GLOBAL Ckpt *)ckpt + im.ckpt_base + (size_t)sv[h] * nck
                                                   : nullptr;
  }
  SyncChain<HuffTable> A, B;
  schain_begin(A, im, tabs, scan, mkp, sv[0], im.lead_bits, active[0], ckv[0], mtp, acm);
  schain_begin(B, im, tabs, scan, mkp, sv[1], im.lead_bits, active[1], ckv[1], mtp, acm);
  schain_run2(A, B, im, tabs, scan, mkp, mtp, acm);
  RangeAcc acc[2] = {A.acc, B.acc};
  ex[t] = active[0] ? A.acc.out : 0u;
  ins[t] = A.in;
  ex[t + 128] = active[1] ? B.acc.out : 0u;
  ins[t + 128] = B.in;
  __syncthreads();
  uint32_t iters = 0;
  for (;;) {
    bool redo[2];
    uint32_t pin[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int q = t + 128 * h;
      redo[h] = active[h] && !head[h] && ins[q] != ex[q - 1];
      pin[h] = redo[h] ? ex[q - 1] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int q = t + 128 * h;
      if (redo[h]) {
        decode_range<false>(im, tabs, scan, mkp, sv[h], pin[h], acc[h], nullptr, ckv[h], true, ex[q], nullptr, mtp,
                            acm, 0u);
        ex[q] = acc[h].out;
        ins[q] = pin[h];
      }
    }
    iters++;
    if (!__syncthreads_or(redo[0] || redo[1])) break;
  }
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int q = t + 128 * h;
    if (active[h] && q > 0) store_sub(subs[im.sub_base + sv[h]], ins[q], ex[q], acc[h]);
  }
  if (t == 0) atomicMax(&flags->sync_iters_max, iters);
  wg_time_store(flags, blockIdx.x, t_start);
}

template <bool STAGE>
__global__ __launch_bounds__(256) void k_huff_fix(const ImageDesc *__restrict__ imgs,
                                                  const WgItem *__restrict__ list,
                                                  const HuffTable *__restrict__ pool,
                                                  SubState *__restrict__ subs, Ckpt *__restrict__ ckpt,
                                                  BatchFlags *flags) {
  extern __shared__ __attribute__((aligned(16))) uint8_t huff_dyn[];
  HuffTable *tabs = (HuffTable *)huff_dyn;
  __shared__ uint32_t ex[kSubPerWg], ins[kSubPerWg];
  if ((flags->debug & kDbgForceChainChange) && blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd(&flags->chain_changed, 1u);
  const WgItem it = list[blockIdx.x];
  const uint32_t s0 = it.item0;
  if (s0 == 0) return;
  const ImageDesc &im = imgs[it.image];
  SubState *base = subs + im.sub_base;
  const uint32_t first_in = base[s0 - 1].out;
  if (base[s0].in == first_in) return;  // boundary already consistent (uniform branch)
  load_tables(tabs, pool, im);
  const int t = threadIdx.x;  // thread t handles s0 + t (t < kUseful)
  const uint32_t s = s0 + t;
  const bool active = t < (int)kUseful && s < im.nsub;
  const uint32_t nck = num_ckpt(im.sub_bits);
  const bool stage = STAGE && im.stage != 0;
  DG_GLOBAL Ckpt *ck =
      (!stage && active && nck && im.ckpt) ? (DG_GLOBAL Ckpt *)ckpt + im.ckpt_base + (size_t)s * nck : nullptr;
  StageCtx sc;
  sc.on = stage && active;
  sc.base = sc.on ? stage_range(im.stage, im.stage_cap, s) : nullptr;
  StageCtx *stg = STAGE ? &sc : nullptr;
  const DG_GLOBAL uint8_t *scan = gp<const uint8_t>(im.ds);
  const DG_GLOBAL uint32_t *mkp = gp<const uint32_t>(im.mk);
  RangeAcc acc = {0, 0, 0, {0, 0, 0}};
  uint32_t orig_out = 0;
  if (active) {
    const SubState &o = base[s];
    orig_out = o.out;
    acc.m = o.m;
    acc.n = o.n;
    acc.dc[0] = o.dc[0];
    acc.dc[1] = o.dc[1];
    acc.dc[2] = o.dc[2];
    ex[t] = o.out;
    ins[t] = o.in;
  } else {
    ex[t] = 0u;
    ins[t] = 0u;
  }
  __syncthreads();
  bool mine = false;
  for (;;) {
    bool redo = active && (t == 0 ? ins[0] != first_in : ins[t] != ex[t - 1]);
    uint32_t pin = redo ? (t == 0 ? first_in : ex[t - 1]) : 0u;
    __syncthreads();
    if (redo) {
      decode_range<false>(im, tabs, scan, mkp, s, pin, acc, nullptr, ck, true, ex[t], stg);
      ex[t] = acc.out;
      ins[t] = pin;
      mine = true;
    }
    if (!__syncthreads_or(redo)) break;
  }
  if (active && mine) {
    store_sub(base[s], ins[t], ex[t], acc, stg);
    bool last = (t == (int)kUseful - 1) && (s + 1 < im.nsub);
    if (last && ex[t] != orig_out) atomicAdd(&flags->chain_changed, 1u);
  }
  if (t == 0) atomicAdd(&flags->fix_count, 1u);
}

// segmented scan element
struct SegAcc {
  uint32_t m, n;
  int32_t d0, d1, d2;
};
__device__ __forceinline__ SegAcc seg_combine(const SegAcc &a, const SegAcc &b) {
  if (b.m) return SegAcc{a.m + b.m, b.n, b.d0, b.d1, b.d2};
  return SegAcc{a.m, a.n + b.n, a.d0 + b.d0, a.d1 + b.d1, a.d2 + b.d2};
}

__global__ __launch_bounds__(256) void k_huff_scan(ImageDesc *__restrict__ imgs,
                                                   const WgItem *__restrict__ list,
                                                   SubState *__restrict__ subs) {
  __shared__ SegAcc sh[kSubPerWg];
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  SubState *base = subs + im.sub_base;
  const int t = threadIdx.x;
  SegAcc carry = {0, 0, 0, 0, 0};
  for (uint32_t c0 = 0; c0 < im.nsub; c0 += kSubPerWg) {
    uint32_t i = c0 + t;
    SegAcc v = {0, 0, 0, 0, 0};
    if (i < im.nsub) v = SegAcc{base[i].m, base[i].n, base[i].dc[0], base[i].dc[1], base[i].dc[2]};
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < kSubPerWg; off <<= 1) {
      SegAcc prev = (t >= off) ? sh[t - off] : SegAcc{0, 0, 0, 0, 0};
      __syncthreads();
      if (t >= off) sh[t] = seg_combine(prev, sh[t]);
      __syncthreads();
    }
    SegAcc ex = (t == 0) ? SegAcc{0, 0, 0, 0, 0} : sh[t - 1];
    SegAcc r = seg_combine(carry, ex);
    if (i < im.nsub) {
      base[i].seg = r.m;
      base[i].nin = r.n;
      base[i].dcin[0] = r.d0;
      base[i].dcin[1] = r.d1;
      base[i].dcin[2] = r.d2;
    }
    carry = seg_combine(carry, sh[kSubPerWg - 1]);
    __syncthreads();
  }
  if (t == 0) {
    uint64_t decoded = im.blocks_per_seg ? (uint64_t)carry.m * im.blocks_per_seg + carry.n : carry.n;
    if (decoded < im.total_blocks) im.status = 2;  // DG_ERR_CORRUPT: truncated entropy data
  }
}

// Per-thread coefficient blocks in LDS, 64 int16 apart with their parts
// swizzled by lane (WriteCtx::sw): the 16-byte zeroing stores and flush loads
// of consecutive lanes cover distinct banks, as the 72-int16 stride of rounds
// 1-4 did, in 32 instead of 36 KiB per workgroup (three workgroups per CU).
constexpr int kBlkStride = 64;

__global__ __launch_bounds__(256) void k_huff_write(ImageDesc *__restrict__ imgs,
                                                    const WgItem *__restrict__ list,
                                                    const HuffTable *__restrict__ pool,
                                                    const SubState *__restrict__ subs, BatchFlags *flags,
                                                    const QuantTable *__restrict__ qpool, uint32_t pair,
                                                    const Ckpt *__restrict__ ckpt) {
  extern __shared__ __attribute__((aligned(16))) uint8_t huff_dyn[];  // im.nslots tables (launch: batch max)
  HuffTable *tabs = (HuffTable *)huff_dyn;
  __shared__ __attribute__((aligned(16))) int16_t blk[kSubPerWg][kBlkStride];
  __shared__ uint32_t wtab[kSubPerWg / 64][128];  // wc_coop_flush tables, one per wave
  __shared__ int32_t qt[3 * 64];                  // fused IDCT: quantisation tables, natural order
  __shared__ uint8_t n2z[64];                     // fused IDCT: natural -> zigzag index
  const uint64_t t_start = wg_clock();
  entropy_setprio(flags);
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  load_tables(tabs, pool, im);
  const bool fused = im.idct_fused != 0;
  if (fused) {
    const int t = threadIdx.x;
    if (t < 64) n2z[kZigzagToNatural[t]] = (uint8_t)t;
    if (t < 3 * 64 && (uint32_t)(t >> 6) < im.ncomp) {
      const DG_GLOBAL uint16_t *q = gp<const uint16_t>((uint64_t)(uintptr_t)qpool[im.qpool[t >> 6]].q);
      qt[t] = q[t & 63];
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  // Split ranges (ImageDesc.ckpt bit 1, option "write_split"): 128 ranges per
  // workgroup, each decoded as two halves by lanes t and t + 64 of a wave
  // pair -- the first half up to the sync pass's half-way checkpoint, the
  // second from the state recorded there, with the blocks and DC sums before
  // it taken from the checkpoint's tail.  Twice the lanes at half the chain:
  // the long 8192-bit ranges that make the sync pass's lead-ins cheap no
  // longer lengthen the write pass.
  const bool split = (im.ckpt & 2u) != 0;
  const uint32_t s = split ? it.item0 + (uint32_t)(t & 63) + ((uint32_t)(t >> 7) << 6) : it.item0 + (uint32_t)t;
  const uint32_t half = split ? ((uint32_t)t >> 6) & 1u : 0u;
  bool run = s < im.nsub;
  uint32_t in = 0, want = 0, a0o = kInf, a1o = kInf;
  SubState ss = {};
  if (run) {
    ss = subs[im.sub_base + s];
    in = ss.in;
    want = ss.out;
    if (split) {
      const uint32_t S = im.sub_bits, mid = s * S + S / 2, kmid = S / 2 / kCkptBits - 1;
      const Ckpt c = ckpt[im.ckpt_base + (size_t)s * num_ckpt(S) + kmid];
      const bool ok = mid < im.ds_bits && im.nmk == 0 && ss.m == 0 && c.m == 0 && st_rel(c.st) < 255u;
      if (!ok) {
        run = half == 0;  // the first lane takes the whole range
      } else if (half == 0) {
        a1o = mid;
        want = c.st;
      } else {
        a0o = mid;
        in = c.st;
        ss.nin += ss.n - c.n;  // blocks started before the checkpoint (tails: checkpoint -> range end)
        ss.dcin[0] += ss.dc[0] - c.dc[0];
        ss.dcin[1] += ss.dc[1] - c.dc[1];
        ss.dcin[2] += ss.dc[2] - c.dc[2];
      }
    }
  }
  if (run) {
    WriteCtx w;
    w.blk = blk[t];
    w.sw = (((uint32_t)t >> 1) & 7u) << 3;
    w.coef = gp<int16_t>(im.coef);
    w.seg = ss.seg;
    w.nin = ss.nin;
    w.pred[0] = ss.dcin[0];
    w.pred[1] = ss.dcin[1];
    w.pred[2] = ss.dcin[2];
    w.blocks_per_seg = im.blocks_per_seg;
    w.total_blocks = im.total_blocks;
    w.cur = -1;
    w.zs = 0;
    w.cnt = (im.ccnt && !fused) ? gp<uint8_t>(im.ccnt) : nullptr;
    w.wave_blk = blk[t & ~63];
    w.stride = kBlkStride;
    w.tab = wtab[t >> 6];
    w.im = fused ? &im : nullptr;
    w.qt = qt;
    w.n2z = n2z;
    w.flags = flags;
    w.img = it.image;
    {  // blocks are all-zero whenever none is open (wc_coop_flush)
      u32x4 *p = (u32x4 *)w.blk;
      const u32x4 zero = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < 8; i++) p[i] = zero;
    }
    RangeAcc acc;
    decode_range<true, HuffTable, true>(im, tabs, gp<const uint8_t>(im.ds), gp<const uint32_t>(im.mk), s, in,
                                        acc, &w, nullptr, false, 0, nullptr, nullptr, 0xFFu, pair, a0o, a1o);
    if (acc.out != want || (s == 0 && (flags->debug & kDbgForceWriteMismatch))) {
      // the write pass left this range in another state than the sync pass
      // proved: the blocks after it are not trustworthy.  The image goes back
      // to the caller's CPU decoder (DG_ERR_UNSUPPORTED) unless it is already
      // known corrupt (k_huff_scan).
      atomicAdd(&flags->write_mismatch, 1u);
      if (imgs[it.image].status == 0) imgs[it.image].status = 1;
    }
  }
  if (flags->wgtime) {
    __syncthreads();
    wg_time_store(flags, flags->wgtime_write + blockIdx.x, t_start);
  }
}

// Decode-once (option "entropy_once"): the blocks from k_huff_sync's staged
// coefficients -- what k_huff_write writes, without decoding the range again.
// One thread per range, its block in LDS as in k_huff_write: blocks are
// started in order (j), carry their DC predictor, and are flushed over the
// zigzag span this range owns (the carried-in block from its entry z, a
// block cut by a marker or by the range end up to that z).
__global__ __launch_bounds__(256) void k_huff_scatter(const ImageDesc *__restrict__ imgs,
                                                      const WgItem *__restrict__ list,
                                                      const SubState *__restrict__ subs) {
  __shared__ __attribute__((aligned(16))) int16_t blk[kSubPerWg][kBlkStride];
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const int t = threadIdx.x;
  const uint32_t s = it.item0 + t;
  if (s >= im.nsub) return;
  const SubState ss = subs[im.sub_base + s];
  WriteCtx w;
  w.blk = blk[t];
  w.coef = gp<int16_t>(im.coef);
  w.seg = ss.seg;
  w.nin = ss.nin;
  w.pred[0] = ss.dcin[0];
  w.pred[1] = ss.dcin[1];
  w.pred[2] = ss.dcin[2];
  w.blocks_per_seg = im.blocks_per_seg;
  w.total_blocks = im.total_blocks;
  w.cur = -1;
  w.zs = 0;
  w.cnt = nullptr;  // dense blocks (decode-once images never get ImageDesc::ccnt)
  if (s * im.sub_bits >= im.ds_bits) return;  // empty trailing range: decodes nothing
  const uint32_t bpm = im.bpm, cbits = im.comp_bits;
  const uint32_t zin = st_z(ss.in);
  uint32_t rn = st_r(ss.in);  // block-in-MCU of the next block to start
  if (zin > 0) {
    wc_begin(w, w.nin > 0 ? wc_index(w, w.nin - 1) : -1, zin);
    rn = rn + 1 == bpm ? 0 : rn + 1;
  }
  uint32_t started = 0, comp = 0;
  auto start_next = [&]() {
    wc_flush(w, 64);  // the open block completed
    comp = (cbits >> (2 * rn)) & 3u;
    rn = rn + 1 == bpm ? 0 : rn + 1;
    wc_begin(w, wc_index(w, w.nin), 0);
    w.nin++;
    w.blk[0] = (int16_t)sel3(w.pred, comp);
    started++;
  };
  const DG_GLOBAL u32x4 *g = (const DG_GLOBAL u32x4 *)stage_range(im.stage, im.stage_cap, s);
  u32x4 grp = {0u, 0u, 0u, 0u};
  for (uint32_t e = 0; e < ss.nent; e++) {
    if ((e & 3u) == 0) grp = g[(size_t)(e >> 2) * 64];
    const uint32_t k = e & 3u;
    const uint32_t v = k == 0 ? grp.x : k == 1 ? grp.y : k == 2 ? grp.z : grp.w;
    if (v & 0x80000000u) {  // RST marker
      const uint32_t zm = (v >> 24) & 63u, j = (v >> 11) & 0x1FFFu;
      while (started < j) start_next();
      wc_flush(w, zm > 0 ? zm : 64);
      if (v & 0x40000000u) {
        w.seg++;
        w.nin = 0;
        w.pred[0] = w.pred[1] = w.pred[2] = 0;
      }
      rn = 0;
      continue;
    }
    const uint32_t zz = v >> 25, j = (v >> 12) & 0x1FFFu;
    const int32_t val = (int32_t)(v << 20) >> 20;
    while (started < j) start_next();
    if (zz == 0) {
      add3(w.pred, comp, val);
      w.blk[0] = (int16_t)sel3(w.pred, comp);
    } else {
      w.blk[zz] = (int16_t)val;
    }
  }
  while (started < ss.nstart) start_next();
  const uint32_t zout = st_z(ss.out);
  wc_flush(w, zout > 0 ? zout : 64);
}

// ------------------------------------------------------------ IDCT

// Pack the low bytes of four values into one dword with explicit v_perm byte
// selects.  Plain shift/or packing of clamped values lets hipcc (ROCm 7.2,
// gfx950) fuse pairs into v_ashr_pk_u8_i32 and then OR the next byte into
// bits 16..23 of that register, whose upper half still holds the old
// accumulator bits: byte 2 of every 4 came out corrupted.  v_perm only takes
// the selected bytes.
__device__ __forceinline__ uint32_t pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  const uint32_t lo = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);  // [b0, b1, 0, 0]
  const uint32_t hi = __builtin_amdgcn_perm(b3, b2, 0x0c0c0400u);  // [b2, b3, 0, 0]
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);               // [b0, b1, b2, b3]
}

// One workgroup = kIdctBlocks consecutive blocks of one block row of one
// component; 8 lanes per block, each lane owning two blocks (slot, slot + 32)
// so two independent 16-byte coefficient loads are in flight per lane and
// the two LDS transposes share their barriers.  Lane `lane` dequantises
// column `lane` in pass 1 (its 8 quant values come from cached loads that
// every block of the wave shares), then runs row `lane` in pass 2.
constexpr uint32_t kIdctBlocks = 64;

__global__ __launch_bounds__(256) void k_idct(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                              const QuantTable *__restrict__ qpool) {
  // Block layout in LDS: element (row r, column c) at r * RS + c, blocks LD
  // dwords apart.  With 4 blocks x 8 lanes per 32-lane bank group, the column
  // accesses of pass 1 (r fixed) and the row reads of pass 2 (c fixed) are
  // conflict-free and the zigzag scatter is at most 2-way (a 64-dword block
  // stride made them 4-, 2- and 3-way).
  constexpr int LD = 72, RS = 9;
  __shared__ int32_t blkv[kIdctBlocks * LD];
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  // item -> (component, block row, chunk of kIdctBlocks blocks)
  uint32_t item = it.item0, c = 0;
  for (; c < im.ncomp; c++) {
    uint32_t ck = (im.cbw[c] + kIdctBlocks - 1) / kIdctBlocks;
    uint32_t n = im.cbh[c] * ck;
    if (item < n) break;
    item -= n;
  }
  const uint32_t ck = (im.cbw[c] + kIdctBlocks - 1) / kIdctBlocks;
  const uint32_t by = item / ck, chunk = item - by * ck;
  const int t = threadIdx.x, slot = t >> 3, lane = t & 7;
  const uint32_t cbw = im.cbw[c];
  const uint32_t bx0 = chunk * kIdctBlocks + slot, bx1 = bx0 + 32;
  const bool v0 = bx0 < cbw, v1 = bx1 < cbw;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(im.coef);
  const uint32_t chc = im.ch[c];
  auto block_index = [&](uint32_t bx) -> uint32_t {
    if (im.ncomp == 1) return by * im.cbw[0] + bx;
    uint32_t my = by / im.cv[c], vy = by - my * im.cv[c];  // uniform
    // per lane: sampling factors are 1..4, and 1 / 2 need no division
    uint32_t mx = chc == 1 ? bx : chc == 2 ? bx >> 1 : bx / chc, hx = bx - mx * chc;
    return (my * im.mcux + mx) * im.bpm + im.cfirst[c] + vy * chc + hx;
  };
  u32x4 r0 = {0, 0, 0, 0}, r1 = {0, 0, 0, 0};
  if (v0) r0 = *(const DG_GLOBAL u32x4 *)(coef + (size_t)block_index(bx0) * 64 + lane * 8);
  if (v1) r1 = *(const DG_GLOBAL u32x4 *)(coef + (size_t)block_index(bx1) * 64 + lane * 8);
  const DG_GLOBAL uint16_t *q = gp<const uint16_t>((uint64_t)(uintptr_t)qpool[im.qpool[c]].q);
  int32_t qc[8];  // column `lane` of the quant table
#pragma unroll
  for (int r = 0; r < 8; r++) qc[r] = q[r * 8 + lane];
  int32_t *bv0 = blkv + slot * LD, *bv1 = blkv + (slot + 32) * LD;
  {
    int16_t a[8], b[8];
    __builtin_memcpy(a, &r0, 16);
    __builtin_memcpy(b, &r1, 16);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int n = kZigzagToNatural[lane * 8 + i];
      const int e = (n >> 3) * RS + (n & 7);
      bv0[e] = a[i];
      bv1[e] = b[i];
    }
  }
  __syncthreads();
  const bool zune = im.sem != 0;  // decode semantics (uniform per workgroup)
  // pass 1: column `lane`, dequantised on the way in
  {
    int32_t v0[8], v1[8], w0[8], w1[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {  // int16 coefficient x uint16 quantiser: 24-bit operands, exact
      v0[r] = __mul24(bv0[r * RS + lane], qc[r]);
      v1[r] = __mul24(bv1[r * RS + lane], qc[r]);
    }
    idct_col(zune, v0, w0);
    idct_col(zune, v1, w1);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; r++) {
      bv0[r * RS + lane] = w0[r];
      bv1[r * RS + lane] = w1[r];
    }
  }
  __syncthreads();
  // pass 2: row `lane`
  const uint32_t pst = cbw * 8;
  DG_GLOBAL uint8_t *plane = gp<uint8_t>(im.plane[c]) + (size_t)(by * 8 + lane) * pst;
  const bool rec = plane_is_rec(im, c);  // uniform per workgroup
  uint32_t pv[2][8];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int32_t *w = (h ? bv1 : bv0) + lane * RS;
    const bool v = h ? v1 : v0;
    int32_t row[8];
    uint32_t px[8];
#pragma unroll
    for (int i = 0; i < 8; i++) row[i] = w[i];
    idct_row(zune, row, px);
    if (rec) {
      crec_clamp((int32_t)crec_lim(im, c) - 1 - (int32_t)((h ? bx1 : bx0) * 8), px, pv[h]);
      continue;
    }
    // pack4, not shifts: shift/or packing of clamped values lets hipcc form
    // v_ashr_pk_u8_i32 and OR the next byte into its stale upper half
    const uint32_t lo = pack4(px[0], px[1], px[2], px[3]), hi = pack4(px[4], px[5], px[6], px[7]);
    if (v) *(DG_GLOBAL u32x2 *)(plane + (size_t)(h ? bx1 : bx0) * 8) = u32x2{lo, hi};
  }
  if (!rec) return;
  // Chroma records (dg_plane.h): the workgroup's 64 blocks are consecutive
  // in the row, so a block's outer edge samples come from its neighbours'
  // edge columns through LDS and both records of a row go out as one 16-byte
  // store; only the first and last block of the chunk hand their edge to
  // (and leave their own to) the neighbouring workgroups.
  __shared__ uint8_t efirst[kIdctBlocks * 8], elast[kIdctBlocks * 8];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int i = slot + 32 * h;
    efirst[i * 8 + lane] = (uint8_t)pv[h][0];
    elast[i * 8 + lane] = (uint8_t)pv[h][7];
  }
  __syncthreads();
  DG_GLOBAL uint8_t *rrow = crec_row(im, c, by * 8 + lane);
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (!(h ? v1 : v0)) continue;
    const int i = slot + 32 * h;
    const uint32_t bx = h ? bx1 : bx0;
    const bool in_l = i > 0, in_r = i + 1 < (int)kIdctBlocks && bx + 1 < cbw;
    const uint32_t l = in_l ? elast[(i - 1) * 8 + lane] : pv[h][0];
    const uint32_t r = in_r ? efirst[(i + 1) * 8 + lane] : pv[h][7];
    store_crec_pair(rrow, bx, cbw, pv[h], l, r, in_l || bx == 0, in_r || bx + 1 == cbw);
  }
}

// Thread-per-block IDCT (option "idct_thread"): one wave = the 64
// consecutive blocks of one block row of one component (the L_IDCT items of
// k_idct), one lane per block.  A lane loads its block's 128 coefficient
// bytes (eight 16-byte loads), dequantises them into 64 registers in natural
// order (the zigzag permutation is a compile-time register renaming), runs
// the 8 column and 8 row transforms in registers and stores its 8 pixel
// rows; the 64 lanes' rows are 512 contiguous bytes of a plane row.  No LDS,
// no barriers, about half k_idct's VALU work per block (k_idct spends 8 lanes
// per block and three LDS round trips on the transposes).  Chroma records
// take their neighbour blocks' edge samples from the adjacent lanes
// (ds_bpermute); only lanes 0 and 63 hand their edges to the neighbouring
// waves by the byte-store protocol of dg_plane.h.
// A workgroup (one wave) takes kIdctItemStride consecutive L_IDCT items in
// turn (the host lists every kIdctItemStride-th item: a quarter of the list
// k_idct needs).  Four waves per workgroup instead measured no better and
// cost 15 VGPRs (109: 4 waves per SIMD).
// Where item `item` of an image puts this lane: component, block row, block
// column, MCU-interleaved block index; false past the image's last item
// (wave-uniform).
struct IdctLoc {
  uint32_t c, by, bx, bidx;
  bool v;  // the lane has a block (bx inside the plane)
};
__device__ __forceinline__ bool idct_t_locate(const ImageDesc &im, uint32_t item, IdctLoc &L) {
  uint32_t c = 0;
  for (; c < im.ncomp; c++) {
    const uint32_t ck = (im.cbw[c] + kIdctBlocks - 1) / kIdctBlocks;
    const uint32_t n = im.cbh[c] * ck;
    if (item < n) break;
    item -= n;
  }
  if (c >= im.ncomp) return false;
  const uint32_t ck = (im.cbw[c] + kIdctBlocks - 1) / kIdctBlocks;
  const uint32_t by = item / ck, chunk = item - by * ck;
  const uint32_t cbw = im.cbw[c];
  const uint32_t bx = chunk * kIdctBlocks + threadIdx.x;
  const uint32_t chc = im.ch[c];
  uint32_t bidx;
  if (im.ncomp == 1) {
    bidx = by * cbw + bx;
  } else {
    const uint32_t my = by / im.cv[c], vy = by - my * im.cv[c];
    const uint32_t mx = chc == 1 ? bx : chc == 2 ? bx >> 1 : bx / chc, hx = bx - mx * chc;
    bidx = (my * im.mcux + mx) * im.bpm + im.cfirst[c] + vy * chc + hx;
  }
  L.c = c;
  L.by = by;
  L.bx = bx;
  L.v = bx < cbw;
  L.bidx = L.v ? bidx : 0u;
  return true;
}

// 16-byte parts of the lane's block to load, as a mask: all 8 for dense
// blocks, the nonzero ones k_huff_write stored for sparse ones
// (ImageDesc::ccnt), none without a block
__device__ __forceinline__ uint32_t idct_t_parts(const ImageDesc &im, const IdctLoc &L) {
  if (!L.v) return 0u;
  if (!im.ccnt) return 0xFFu;
  return gp<const uint8_t>(im.ccnt)[L.bidx];
}

__device__ __forceinline__ void idct_t_item(const ImageDesc &im, const IdctLoc &L, const u32x4 w[8],
                                            const QuantTable *__restrict__ qpool);

__global__ __launch_bounds__(64) void k_idct_t(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                              const QuantTable *__restrict__ qpool) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  // Sparse blocks: the part count of the next item's block is loaded while
  // this item transforms, so the count -> parts dependency costs one memory
  // round trip per workgroup, not one per item.
  IdctLoc L;
  bool ok = idct_t_locate(im, it.item0, L);
  uint32_t np = ok ? idct_t_parts(im, L) : 0u;
#pragma nounroll
  for (uint32_t k = 0; k < kIdctItemStride && ok; k++) {
    u32x4 w[8];
    const DG_GLOBAL u32x4 *src = (const DG_GLOBAL u32x4 *)(gp<const int16_t>(im.coef) + (size_t)L.bidx * 64);
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) w[i] = (np >> i) & 1u ? src[i] : u32x4{0, 0, 0, 0};
    IdctLoc N;
    const bool nok = k + 1 < kIdctItemStride && idct_t_locate(im, it.item0 + k + 1, N);
    const uint32_t nnp = nok ? idct_t_parts(im, N) : 0u;
    idct_t_item(im, L, w, qpool);
    L = N;
    ok = nok;
    np = nnp;
  }
}

__device__ __forceinline__ void idct_t_item(const ImageDesc &im, const IdctLoc &L, const u32x4 w[8],
                                            const QuantTable *__restrict__ qpool) {
  const uint32_t c = L.c, by = L.by, bx = L.bx;
  const bool v = L.v;
  const uint32_t lane = threadIdx.x, cbw = im.cbw[c];
  // Decode semantics as a runtime flag: with it as a template constant the
  // whole block's transforms become one straight-line region and the
  // scheduler interleaves all eight columns (185 VGPRs, 2 waves per SIMD);
  // the per-transform branch keeps it at 94.
  const bool zune = im.sem != 0;
  const DG_GLOBAL uint16_t *q = gp<const uint16_t>((uint64_t)(uintptr_t)qpool[im.qpool[c]].q);
  int32_t x[64];
  {
#pragma unroll
    for (int k = 0; k < 64; k++) {
      const uint32_t word = w[k >> 3][(k >> 1) & 3];
      const int32_t z = (int32_t)(int16_t)(k & 1 ? word >> 16 : word & 0xFFFFu);
      const int nat = kZigzagToNatural[k];
      x[nat] = __mul24(z, (int32_t)q[nat]);  // int16 x uint16: 24-bit operands, exact
    }
  }
#pragma unroll
  for (int col = 0; col < 8; col++) {
    int32_t in[8], o[8];
#pragma unroll
    for (int r = 0; r < 8; r++) in[r] = x[r * 8 + col];
    idct_col(zune, in, o);
#pragma unroll
    for (int r = 0; r < 8; r++) x[r * 8 + col] = o[r];
  }
  const bool rec = plane_is_rec(im, c);
  const int32_t e = rec ? (int32_t)crec_lim(im, c) - 1 - (int32_t)(bx * 8) : 7;
  DG_GLOBAL uint8_t *plane = gp<uint8_t>(im.plane[c]);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint32_t px[8];
    idct_row(zune, x + r * 8, px);
    const uint32_t y = by * 8 + (uint32_t)r;
    if (!rec) {
      if (v)
        *(DG_GLOBAL u32x2 *)(plane + (size_t)y * (cbw * 8) + bx * 8) =
            u32x2{pack4(px[0], px[1], px[2], px[3]), pack4(px[4], px[5], px[6], px[7])};
      continue;
    }
    uint32_t vv[8];
    crec_clamp(e, px, vv);
    // neighbours' edge columns from the adjacent lanes (every lane takes part)
    const uint32_t l = (uint32_t)__shfl_up((int)vv[7], 1), rr = (uint32_t)__shfl_down((int)vv[0], 1);
    if (v) {
      const bool have_l = lane > 0 || bx == 0, have_r = (lane + 1 < 64u && bx + 1 < cbw) || bx + 1 == cbw;
      store_crec_pair(crec_row(im, c, y), bx, cbw, vv, lane > 0 ? l : vv[0], bx + 1 < cbw ? rr : vv[7], have_l,
                      have_r);
    }
  }
}


// Fused-IDCT leftovers (option "idct_fused"): the blocks k_huff_write could
// not turn into pixels itself -- a block completed by a range that did not
// start it (its first coefficients came from the previous range), or
// flushed when fewer than 8 lanes were active -- were written as
// coefficients and listed in BatchFlags::idct_list.  8 lanes per block, 32
// blocks per workgroup round, grid-strided over the device-side count.
__global__ __launch_bounds__(256) void k_idct_list(const ImageDesc *__restrict__ imgs,
                                                   const QuantTable *__restrict__ qpool,
                                                   const BatchFlags *__restrict__ flags) {
  constexpr int LD = 72, RS = 9;
  __shared__ int32_t blkv[32 * LD];
  const uint32_t n = flags->idct_late < flags->idct_cap ? flags->idct_late : flags->idct_cap;
  const DG_GLOBAL uint32_t *list = gp<const uint32_t>(flags->idct_list);
  const int t = threadIdx.x, slot = t >> 3, lane = t & 7;
  int32_t *bv = blkv + slot * LD;
  for (uint32_t base = blockIdx.x * 32; base < n; base += gridDim.x * 32) {  // uniform per workgroup
    const uint32_t e = base + (uint32_t)slot;
    const bool act = e < n;
    const uint32_t ii = act ? list[2 * e] : 0u, idx = act ? list[2 * e + 1] : 0u;
    const ImageDesc &im = imgs[ii];
    uint32_t c = 0, by = 0, bx = 0;
    if (act) block_pos(im, idx, c, by, bx);
    if (act) {
      const u32x4 r0 = *(const DG_GLOBAL u32x4 *)(gp<const int16_t>(im.coef) + (size_t)idx * 64 + lane * 8);
      int16_t a[8];
      __builtin_memcpy(a, &r0, 16);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int nn = kZigzagToNatural[lane * 8 + i];
        bv[(nn >> 3) * RS + (nn & 7)] = a[i];
      }
    }
    __syncthreads();
    int32_t w[8];
    if (act) {
      const DG_GLOBAL uint16_t *q = gp<const uint16_t>((uint64_t)(uintptr_t)qpool[im.qpool[c]].q);
      int32_t v[8];
#pragma unroll
      for (int r = 0; r < 8; r++) v[r] = bv[r * RS + lane] * (int32_t)q[r * 8 + lane];
      idct_col(im.sem != 0, v, w);
    }
    __syncthreads();
    if (act) {
#pragma unroll
      for (int r = 0; r < 8; r++) bv[r * RS + lane] = w[r];
    }
    __syncthreads();
    if (act) {
      int32_t row[8];
      uint32_t px[8];
#pragma unroll
      for (int i = 0; i < 8; i++) row[i] = bv[lane * RS + i];
      idct_row(im.sem != 0, row, px);
      store_plane_row8(im, c, by * 8 + lane, bx, px);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ colour

// 8 consecutive upsampled samples of component plane `pl` at row y, columns
// x0..x0+7 (x0 a multiple of 8), with libjpeg's fancy filters (see
// upsample_at, which this vectorises: one aligned load per source row plus
// the two edge samples instead of four byte loads per pixel).
// Row offsets use 24-bit multiplies (full rate, v_mul_lo_u32 is quarter rate):
// the host keeps every JPEG plane below 4 GiB (pipeline.cpp, plan_image).
template <class P>
__device__ __forceinline__ void upsample8(P pl, uint32_t stride, uint32_t hr, uint32_t vr,
                                          uint32_t dsw, uint32_t dsh, uint32_t x0, uint32_t y, int32_t o[8],
                                          bool rec = false) {
  if (rec) {  // chroma records (dg_plane.h): six clamped columns per row in one load, no edge cases
    const uint32_t c0 = x0 >> 1;
    int32_t cs[6];
    const bool fancy = dsw > 2;
    if (vr == 1 || !fancy) {
      load_crec6(pl, stride, vr == 1 ? y : y >> 1, c0, cs);
      if (!fancy) {
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = cs[1 + (k >> 1)];
        return;
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int32_t a = cs[k + 1] * 3;
        o[2 * k] = (a + cs[k] + 1) >> 2;
        o[2 * k + 1] = (a + cs[k + 2] + 2) >> 2;
      }
      return;
    }
    const uint32_t r = y >> 1;
    int32_t rn = (y & 1) ? (int32_t)r + 1 : (int32_t)r - 1;
    rn = rn < 0 ? 0 : (rn > (int32_t)dsh - 1 ? (int32_t)dsh - 1 : rn);
    int32_t fr[6];
    load_crec6(pl, stride, r, c0, cs);
    load_crec6(pl, stride, (uint32_t)rn, c0, fr);
#pragma unroll
    for (int k = 0; k < 6; k++) cs[k] = cs[k] * 3 + fr[k];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[2 * k] = (cs[k + 1] * 3 + cs[k] + 8) >> 4;
      o[2 * k + 1] = (cs[k + 1] * 3 + cs[k + 2] + 7) >> 4;
    }
    return;
  }
  if (hr == 1) {  // 4:4:4 component (vr is 1 too for the supported samplings)
    u32x2 v = *(const DG_GLOBAL u32x2 *)(pl + (size_t)__umul24(y, stride) + x0);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[k] = (v.x >> (8 * k)) & 0xFF;
      o[k + 4] = (v.y >> (8 * k)) & 0xFF;
    }
    return;
  }
  const uint32_t c0 = x0 >> 1;  // multiple of 4
  const bool fancy = dsw > 2;
  int32_t cs[6];                // column sums (or plain samples for h2v1) at c0-1 .. c0+4
  const uint32_t cl = c0 > 0 ? c0 - 1 : 0, cr = c0 + 4 < dsw ? c0 + 4 : dsw - 1;
  if (vr == 1) {
    P in = pl + (size_t)__umul24(y, stride);
    uint32_t v = *(const DG_GLOBAL uint32_t *)(in + c0);
    cs[0] = in[cl];
#pragma unroll
    for (int k = 0; k < 4; k++) cs[k + 1] = (v >> (8 * k)) & 0xFF;
    cs[5] = in[cr];
    // clamp interior samples past the downsampled width (replicate the edge)
    if (c0 + 5 > dsw) {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (c0 + k >= dsw) cs[k + 1] = cs[dsw - c0];
    }
    if (!fancy) {
#pragma unroll
      for (int k = 0; k < 8; k++) o[k] = cs[1 + (k >> 1)];
      return;
    }
    if (c0 + 5 <= dsw) {  // interior lanes: every right neighbour exists
#pragma unroll
      for (int k = 0; k < 4; k++) {
        int32_t a = cs[k + 1] * 3;
        o[2 * k] = (a + cs[k] + 1) >> 2;
        o[2 * k + 1] = (a + cs[k + 2] + 2) >> 2;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        int32_t a = cs[k + 1] * 3;
        int32_t nl = (c0 + k + 1 < dsw) ? cs[k + 2] : cs[k + 1];
        o[2 * k] = (a + cs[k] + 1) >> 2;
        o[2 * k + 1] = (a + nl + 2) >> 2;
      }
    }
    if (c0 == 0) o[0] = (cs[1] * 3 + cs[1] + 1) >> 2;
    return;
  }
  // h2v2
  const uint32_t r = y >> 1;
  if (!fancy) {
    P in = pl + (size_t)__umul24(r, stride);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t c = c0 + (k >> 1);
      o[k] = in[c < dsw ? c : dsw - 1];
    }
    return;
  }
  int32_t rn = (y & 1) ? (int32_t)r + 1 : (int32_t)r - 1;
  rn = rn < 0 ? 0 : (rn > (int32_t)dsh - 1 ? (int32_t)dsh - 1 : rn);
  P i0 = pl + (size_t)__umul24(r, stride);
  P i1 = pl + (size_t)__umul24((uint32_t)rn, stride);
  uint32_t v0 = *(const DG_GLOBAL uint32_t *)(i0 + c0), v1 = *(const DG_GLOBAL uint32_t *)(i1 + c0);
  cs[0] = i0[cl] * 3 + i1[cl];
#pragma unroll
  for (int k = 0; k < 4; k++) cs[k + 1] = (int32_t)((v0 >> (8 * k)) & 0xFF) * 3 + (int32_t)((v1 >> (8 * k)) & 0xFF);
  cs[5] = i0[cr] * 3 + i1[cr];
  if (c0 + 5 <= dsw) {  // interior lanes: no clamping, every right neighbour exists
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[2 * k] = (cs[k + 1] * 3 + cs[k] + 8) >> 4;
      o[2 * k + 1] = (cs[k + 1] * 3 + cs[k + 2] + 7) >> 4;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (c0 + k >= dsw) cs[k + 1] = cs[dsw - c0];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int32_t nl = (c0 + k + 1 < dsw) ? cs[k + 2] : cs[k + 1];
      o[2 * k] = (cs[k + 1] * 3 + cs[k] + 8) >> 4;
      o[2 * k + 1] = (cs[k + 1] * 3 + nl + 7) >> 4;
    }
  }
}

// zune-jpeg upsampling (option "decode_semantics" = 1; oracle upsample_row_zune):
// over the MCU-padded rows (n = stride samples, ph padded rows), h2v2 first
// vertically (3 * near + far + 2) >> 2 with the row itself past either end,
// then horizontally (3 * a + b + 2) >> 2 on both phases; out[0] = in[0],
// the last pair is ((3 * in[n-2] + in[n-1] + 2) >> 2, in[n-1]).
template <class P>
__device__ __forceinline__ void upsample8_zune(P pl, uint32_t stride, uint32_t hr, uint32_t vr, uint32_t ph,
                                               uint32_t x0, uint32_t y, int32_t o[8], bool rec = false) {
  if (rec) {  // chroma records (dg_plane.h), columns clamped to [0, n-1]
    const uint32_t n = stride, c0 = x0 >> 1;
    int32_t cs[6];
    if (vr == 1) {
      load_crec6(pl, stride, y, c0, cs);
    } else {
      const uint32_t r = y >> 1;
      const uint32_t rn = (y & 1) ? (r + 1 < ph ? r + 1 : r) : (r > 0 ? r - 1 : 0);
      int32_t fr[6];
      load_crec6(pl, stride, r, c0, cs);
      load_crec6(pl, stride, rn, c0, fr);
#pragma unroll
      for (int k = 0; k < 6; k++) cs[k] = (3 * cs[k] + 2 + fr[k]) >> 2;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {  // column 0: cs[0] == cs[1], so the even output is cs[1] as zune's
      const int32_t a = 3 * cs[k + 1] + 2;
      int32_t ev = (a + cs[k]) >> 2, od = (a + cs[k + 2]) >> 2;
      if (c0 + (uint32_t)k + 1 == n) {
        ev = (3 * cs[k] + cs[k + 1] + 2) >> 2;
        od = cs[k + 1];
      }
      o[2 * k] = ev;
      o[2 * k + 1] = od;
    }
    return;
  }
  if (hr == 1) {
    u32x2 v = *(const DG_GLOBAL u32x2 *)(pl + (size_t)__umul24(y, stride) + x0);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[k] = (v.x >> (8 * k)) & 0xFF;
      o[k + 4] = (v.y >> (8 * k)) & 0xFF;
    }
    return;
  }
  const uint32_t n = stride, c0 = x0 >> 1;  // c0 + 3 <= n - 1 (x0 + 8 <= 2n)
  const uint32_t cl = c0 > 0 ? c0 - 1 : 0, cr = c0 + 4 < n ? c0 + 4 : n - 1;
  int32_t cs[6];  // (vertically upsampled) samples at columns c0-1 .. c0+4, clamped
  if (vr == 1) {
    P in = pl + (size_t)__umul24(y, stride);
    const uint32_t v = *(const DG_GLOBAL uint32_t *)(in + c0);
    cs[0] = in[cl];
#pragma unroll
    for (int k = 0; k < 4; k++) cs[k + 1] = (v >> (8 * k)) & 0xFF;
    cs[5] = in[cr];
  } else {
    const uint32_t r = y >> 1;
    const uint32_t rn = (y & 1) ? (r + 1 < ph ? r + 1 : r) : (r > 0 ? r - 1 : 0);
    P i0 = pl + (size_t)__umul24(r, stride);
    P i1 = pl + (size_t)__umul24(rn, stride);
    const uint32_t v0 = *(const DG_GLOBAL uint32_t *)(i0 + c0), v1 = *(const DG_GLOBAL uint32_t *)(i1 + c0);
    cs[0] = (3 * (int32_t)i0[cl] + 2 + (int32_t)i1[cl]) >> 2;
#pragma unroll
    for (int k = 0; k < 4; k++)
      cs[k + 1] = (3 * (int32_t)((v0 >> (8 * k)) & 0xFF) + 2 + (int32_t)((v1 >> (8 * k)) & 0xFF)) >> 2;
    cs[5] = (3 * (int32_t)i0[cr] + 2 + (int32_t)i1[cr]) >> 2;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t i = c0 + (uint32_t)k;
    const int32_t a = 3 * cs[k + 1] + 2;
    int32_t ev = (a + cs[k]) >> 2, od = (a + cs[k + 2]) >> 2;
    if (i == 0) ev = cs[1];
    if (i + 1 == n) {
      ev = (3 * cs[k] + cs[k + 1] + 2) >> 2;
      od = cs[k + 1];
    }
    o[2 * k] = ev;
    o[2 * k + 1] = od;
  }
}

// the three components of 8 pixels at (x0.., y), upsampled per the image's decode semantics
__device__ __forceinline__ void upsample_ycc8(const ImageDesc &im, uint32_t x0, uint32_t y, int32_t Y[8],
                                             int32_t Cb[8], int32_t Cr[8]) {
  if (im.sem) {
    upsample8_zune(gp<const uint8_t>(im.plane[0]), im.cbw[0] * 8, im.hmax / im.ch[0], im.vmax / im.cv[0],
                   im.cbh[0] * 8, x0, y, Y, plane_is_rec(im, 0));
    upsample8_zune(gp<const uint8_t>(im.plane[1]), im.cbw[1] * 8, im.hmax / im.ch[1], im.vmax / im.cv[1],
                   im.cbh[1] * 8, x0, y, Cb, plane_is_rec(im, 1));
    upsample8_zune(gp<const uint8_t>(im.plane[2]), im.cbw[2] * 8, im.hmax / im.ch[2], im.vmax / im.cv[2],
                   im.cbh[2] * 8, x0, y, Cr, plane_is_rec(im, 2));
    return;
  }
  upsample8(gp<const uint8_t>(im.plane[0]), im.cbw[0] * 8, im.hmax / im.ch[0], im.vmax / im.cv[0], im.cdsw[0],
            im.cdsh[0], x0, y, Y, plane_is_rec(im, 0));
  upsample8(gp<const uint8_t>(im.plane[1]), im.cbw[1] * 8, im.hmax / im.ch[1], im.vmax / im.cv[1], im.cdsw[1],
            im.cdsh[1], x0, y, Cb, plane_is_rec(im, 1));
  upsample8(gp<const uint8_t>(im.plane[2]), im.cbw[2] * 8, im.hmax / im.ch[2], im.vmax / im.cv[2], im.cdsw[2],
            im.cdsh[2], x0, y, Cr, plane_is_rec(im, 2));
}

__device__ __forceinline__ void ycc_px(const ImageDesc &im, int32_t y, int32_t cb, int32_t cr, uint8_t &r,
                                       uint8_t &g, uint8_t &b) {
  if (im.colorspace == CS_RGB) {
    r = (uint8_t)y;
    g = (uint8_t)cb;
    b = (uint8_t)cr;
  } else if (im.sem) {
    ycc_to_rgb_zune(y, cb, cr, r, g, b);
  } else {
    ycc_to_rgb(y, cb, cr, r, g, b);
  }
}

__global__ __launch_bounds__(256) void k_color(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const uint32_t ow = (im.width + 7) / 8;  // octets per row
  const uint32_t q = it.item0 + threadIdx.x;
  if (q >= ow * im.height) return;
  const uint32_t y = q / ow, x0 = (q - y * ow) * 8;
  int32_t Y[8], Cb[8], Cr[8];
  upsample_ycc8(im, x0, y, Y, Cb, Cr);
  uint32_t w[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint8_t r, g, b;
    ycc_px(im, Y[k], Cb[k], Cr[k], r, g, b);
    const int o = 3 * k;
    w[o >> 2] |= (uint32_t)r << (8 * (o & 3));
    w[(o + 1) >> 2] |= (uint32_t)g << (8 * ((o + 1) & 3));
    w[(o + 2) >> 2] |= (uint32_t)b << (8 * ((o + 2) & 3));
  }
  DG_GLOBAL uint8_t *dst = gp<uint8_t>(im.pix) + (size_t)y * im.pix_stride + x0 * 3;
  if (x0 + 8 <= im.width) {
    DG_GLOBAL u32x2 *d = (DG_GLOBAL u32x2 *)dst;  // x0*3 is a multiple of 24, pix_stride of 16
    d[0] = u32x2{w[0], w[1]};
    d[1] = u32x2{w[2], w[3]};
    d[2] = u32x2{w[4], w[5]};
  } else {
    const uint32_t n = (im.width - x0) * 3;
    for (uint32_t i = 0; i < n; i++) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}

// ------------------------------------------------------------ resize

__device__ __forceinline__ uint8_t clip_shift(int32_t acc, int32_t prec) {
  int32_t v = acc >> prec;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ __launch_bounds__(256) void k_coeffs(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ double red[256];
  const WgItem it = list[blockIdx.x];
  ResizePass &ps = imgs[it.image].pass[it.item0];
  const int t = threadIdx.x;
  const double in0 = ps.in0, in1 = ps.in1;
  const uint32_t out_size = ps.out_size, in_size = ps.in_size, ksize = ps.ksize;
  const double scale = (in1 - in0) / (double)out_size;
  const double filter_scale = scale > 1.0 ? scale : 1.0;
  const double support = 3.0 * filter_scale;
  const double recip = 1.0 / filter_scale;
  DG_GLOBAL int32_t *bounds = gp<int32_t>(ps.bounds);  // {start, size} per output
  DG_GLOBAL int16_t *coef = gp<int16_t>(ps.coef);
  // Each tap's Lanczos value is evaluated twice (the sum, then the
  // quantisation), not four times: the largest normalised weight of an output
  // is its largest (smallest, for a negative sum) raw weight divided by the
  // sum -- division by one value is monotone in IEEE arithmetic, so this is
  // exactly the max of the quotients -- and each output's sum waits for the
  // second loop in the first 8 bytes of its own coefficient row (ksize >= 7
  // taps of 2 bytes; the same thread owns output o in both loops).
  double maxw = 0.0;
  for (uint32_t o = t; o < out_size; o += 256) {
    // fast_image_resize precompute_coefficients for output o (see fir_weights)
    double center = in0 + ((double)o + 0.5) * scale;
    double fl = floor(center - support), cl = ceil(center + support);
    int32_t xmin = fl < 0.0 ? 0 : (int32_t)fl;
    int32_t xmax = cl > (double)in_size ? (int32_t)in_size : (int32_t)cl;
    double c = center - 0.5, ww = 0.0, vhi = -INFINITY, vlo = INFINITY;
    int32_t first = -1, last = -1;
    for (int32_t x = xmin; x < xmax; x++) {
      double v = lanczos3(((double)x - c) * recip);
      if (v != 0.0) {
        if (first < 0) first = x;
        last = x;
        vhi = v > vhi ? v : vhi;
        vlo = v < vlo ? v : vlo;
      }
      ww += v;
    }
    int32_t st = first < 0 ? xmax : first;
    int32_t n = first < 0 ? 0 : last - first + 1;
    bounds[2 * o] = st;
    bounds[2 * o + 1] = n;
    {
      const uint64_t bits = __builtin_bit_cast(uint64_t, ww);
      DG_GLOBAL uint16_t *kw = (DG_GLOBAL uint16_t *)(coef + (size_t)o * ksize);
#pragma unroll
      for (int q = 0; q < 4; q++) kw[q] = (uint16_t)(bits >> (16 * q));
    }
    if (n > 0) {  // the taps [st, st + n) hold every nonzero weight; zeros inside it are 0 / ww = 0
      const double hi = ww > 0.0 ? vhi / ww : ww < 0.0 ? vlo / ww : vhi;
      const double cand = hi > 0.0 ? hi : 0.0;  // a zero weight inside the window still compares
      if (cand > maxw) maxw = cand;
    }
  }
  red[t] = maxw;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] = red[t] > red[t + off] ? red[t] : red[t + off];
    __syncthreads();
  }
  const int32_t precision = fir_precision(red[0]);
  if (t == 0) ps.precision = precision;
  for (uint32_t o = t; o < out_size; o += 256) {
    double center = in0 + ((double)o + 0.5) * scale;
    double c = center - 0.5;
    DG_GLOBAL int16_t *k = coef + (size_t)o * ksize;
    uint64_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) bits |= (uint64_t)(uint16_t)k[q] << (16 * q);
    const double ww = __builtin_bit_cast(double, bits);
    const int32_t st = bounds[2 * o], n = bounds[2 * o + 1];
    for (int32_t i = n; i < 4; i++) k[i] = 0;  // taps past n keep no stale sum bits
    for (int32_t i = 0; i < n; i++) {
      double v = lanczos3(((double)(st + i) - c) * recip);
      if (ww != 0.0) v /= ww;
      k[i] = fir_quant(v, precision);
    }
  }
}


// Horizontal pass: one workgroup = one output row x kResizeTile output
// columns.  The source row segment those columns read is staged in LDS with
// coalesced dword loads, then each thread convolves 2 output pixels from LDS.
constexpr uint32_t kResizeTile = 512;

// One output pixel of a horizontal pass: C channels, n taps from s[off...].
template <class P>
__device__ __forceinline__ void hconv(P s, uint32_t off, int32_t n, const DG_GLOBAL int16_t *k, uint32_t C,
                                      int32_t prec, DG_GLOBAL uint8_t *dst) {
  const int32_t bias = 1 << (prec - 1);
  if (C == 3) {
    int32_t a0 = bias, a1 = bias, a2 = bias;
    for (int32_t i = 0; i < n; i++) {
      const int32_t w = k[i];
      const uint32_t o = off + 3 * (uint32_t)i;
      a0 += (int32_t)s[o] * w;
      a1 += (int32_t)s[o + 1] * w;
      a2 += (int32_t)s[o + 2] * w;
    }
    dst[0] = clip_shift(a0, prec);
    dst[1] = clip_shift(a1, prec);
    dst[2] = clip_shift(a2, prec);
  } else {
    for (uint32_t ch = 0; ch < C; ch++) {
      int32_t a = bias;
      for (int32_t i = 0; i < n; i++) a += (int32_t)s[off + (uint32_t)i * C + ch] * (int32_t)k[i];
      dst[ch] = clip_shift(a, prec);
    }
  }
}
constexpr uint32_t kResizeSeg = 24576;  // LDS bytes for the staged source segment

__global__ __launch_bounds__(256) void k_resize_h(const ImageDesc *__restrict__ imgs,
                                                  const WgItem *__restrict__ list, int stage_flags) {
  __shared__ __attribute__((aligned(16))) uint8_t seg[kResizeSeg + 16];
  const int stage = stage_flags & 0xFF;
  const WgItem it = list[blockIdx.x];
  const ResizePass &ps = imgs[it.image].pass[stage];
  const uint32_t tiles = (ps.width + kResizeTile - 1) / kResizeTile;
  const uint32_t y = it.item0 / tiles, tile = it.item0 - y * tiles;
  if (y >= ps.rows) return;
  const uint32_t x0 = tile * kResizeTile;
  const uint32_t x1 = x0 + kResizeTile < ps.width ? x0 + kResizeTile : ps.width;
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;  // {start, size} per output
  const uint32_t C = ps.C;
  // source bytes [sb, se) of the tile (min/max: trimmed starts are not monotone)
  __shared__ uint32_t ext[2];
  if (threadIdx.x == 0) {
    ext[0] = 0xFFFFFFFFu;
    ext[1] = 0;
  }
  __syncthreads();
  for (uint32_t x = x0 + threadIdx.x; x < x1; x += 256) {
    atomicMin(&ext[0], (uint32_t)bounds[2 * x]);
    atomicMax(&ext[1], (uint32_t)(bounds[2 * x] + bounds[2 * x + 1]));
  }
  __syncthreads();
  const uint32_t sb = ext[0] * C;
  const uint32_t se = ext[1] * C;
  const DG_GLOBAL uint8_t *srow = gp<const uint8_t>(ps.src) + (size_t)(ps.row0 + y) * ps.src_stride;
  const bool staged = se - sb + 8 <= kResizeSeg && !(stage_flags & 0x100);
  const uint32_t a0 = sb & ~3u;  // dword-aligned start (src_stride is a multiple of 4)
  if (staged) {
    const uint32_t nw = (se - a0 + 3) >> 2;
    const DG_GLOBAL uint32_t *s4 = (const DG_GLOBAL uint32_t *)(srow + a0);
    uint32_t *d4 = (uint32_t *)seg;
    for (uint32_t i = threadIdx.x; i < nw; i += 256) d4[i] = s4[i];
  }
  __syncthreads();
  DG_GLOBAL uint8_t *drow = gp<uint8_t>(ps.dst) + (size_t)y * ps.dst_stride;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ps.ksize;
  const int32_t prec = ps.precision;
  if (staged) {
    for (uint32_t x = x0 + threadIdx.x; x < x1; x += 256)
      hconv(seg, (uint32_t)bounds[2 * x] * C - a0, bounds[2 * x + 1], coef + (size_t)x * ps.ksize, C,
            prec, drow + (size_t)x * C);
  } else {  // extreme downscale: segment larger than LDS, read the row directly
    for (uint32_t x = x0 + threadIdx.x; x < x1; x += 256)
      hconv(srow, (uint32_t)bounds[2 * x] * C, bounds[2 * x + 1], coef + (size_t)x * ps.ksize, C,
            prec, drow + (size_t)x * C);
  }
}

// Blocks b and b+8 land on the same XCD (round-robin placement, speed only):
// map them to consecutive work items so each XCD's L2 sees a contiguous run
// of rows of one image instead of every eighth row of all of them.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t per = n >> 3, rem = n & 7, x = b & 7, l = b >> 3;
  return x * per + (x < rem ? x : rem) + l;
}

// ---- band H pass
//
// One workgroup = kHBandCols output columns x kHBandRows rows.  Phase 1 stages
// the source segment of every row of the band in LDS (one dword per pixel,
// channels in bytes 0..3) with all 256 threads; phase 2 has each thread
// convolve one output column for kHBandRows/2 rows with the column's Lanczos
// weights held in registers (one ds_read_b32 per tap); phase 3 stores the
// band's rows with 16-byte writes.  The fill either copies interleaved bytes
// (C = 1..4) or — for the first pass of a colour JPEG — upsamples and
// colour-converts straight from the Y/Cb/Cr planes, so the full-size RGB
// image never exists in HBM.
constexpr uint32_t kHSegStride = kHSegPx + 8;
// Fused first H + V pass (k_resize_hv): the H rows a workgroup's V outputs
// need stay in an LDS ring of kHVRing rows instead of going through HBM.
constexpr uint32_t kHVRing = 32;                  // >= V taps + one band of 8 rows
constexpr uint32_t kHVSegStride = kHVSegPx + 8;  // (kHVSegPx, kHVTapsMax, kHVRows: dg_types.h)
constexpr uint32_t kHVOut = 8;                    // k_resize_hv: V rows produced per round

// job j of the fill: 8 source pixels from the planes, p0 % 8 == 0
__device__ __forceinline__ void hcolor8(const ImageDesc &im, uint32_t y, uint32_t x0, uint32_t v[8]) {
  int32_t Y[8], Cb[8], Cr[8];
  upsample_ycc8(im, x0, y, Y, Cb, Cr);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint8_t r, g, b;
    ycc_px(im, Y[k], Cb[k], Cr[k], r, g, b);
    v[k] = (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16);
  }
}
__device__ __forceinline__ void hfill_color8(const ImageDesc &im, uint32_t y, uint32_t x0, uint32_t *d) {
  uint32_t v[8];
  hcolor8(im, y, x0, v);
  u32x4 *d4 = (u32x4 *)d;
  d4[0] = u32x4{v[0], v[1], v[2], v[3]};
  d4[1] = u32x4{v[4], v[5], v[6], v[7]};
}

// Fill classes of the fused colour fill: the common JPEG layouts get a fill
// specialised at compile time (no per-pixel branches on sampling, semantics,
// record format or colour space, no edge clamping: the chroma records carry
// their clamped edges); everything else takes the generic hfill_color8.
// Chosen once per workgroup (uniform per image).
enum FillClass : int {
  FC_GENERIC = 0,
  FC_420 = 1, FC_420_Z = 2,  // Y h2v2, Cb/Cr h1v1 as chroma records; libjpeg fancy / zune
  FC_422 = 3, FC_422_Z = 4,  // Y h2v1, Cb/Cr h1v1 as chroma records
  FC_444 = 5, FC_444_Z = 6,  // all components at full rate (plain planes)
};

__device__ __forceinline__ int fill_class(const ImageDesc &im) {
  if (im.ncomp != 3 || im.colorspace != CS_YCC) return FC_GENERIC;
  const bool z = im.sem != 0;
  if (im.ch[0] == 1 && im.cv[0] == 1 && im.ch[1] == 1 && im.cv[1] == 1 && im.ch[2] == 1 && im.cv[2] == 1 &&
      im.crec == 0)
    return z ? FC_444_Z : FC_444;
  if (im.ch[0] != 2 || im.ch[1] != 1 || im.cv[1] != 1 || im.ch[2] != 1 || im.cv[2] != 1 || im.crec != 6u)
    return FC_GENERIC;
  if (!z && (im.cdsw[1] <= 2 || im.cdsw[2] <= 2)) return FC_GENERIC;  // libjpeg's box filter for tiny widths
  if (im.cv[0] == 2) return z ? FC_420_Z : FC_420;
  if (im.cv[0] == 1) return z ? FC_422_Z : FC_422;
  return FC_GENERIC;
}

// The raw plane words one octet of a specialised fill reads: luma, and the
// chroma (records, or plain samples for 4:4:4) of the near (0) and far (1)
// chroma rows.  Loading them is split from the arithmetic (hcolor_fc8) so
// the band kernel can issue the next band's loads before the convolution.
struct FillRaw {
  u32x2 y, b0, r0, b1, r1;
};

template <int FC>
__device__ __forceinline__ FillRaw hload_fc8(const ImageDesc &im, uint32_t y, uint32_t x0) {
  constexpr bool Z = FC == FC_420_Z || FC == FC_422_Z || FC == FC_444_Z;
  constexpr int SS = (FC == FC_420 || FC == FC_420_Z) ? 2 : (FC == FC_422 || FC == FC_422_Z) ? 1 : 0;
  const DG_GLOBAL uint8_t *pY = gp<const uint8_t>(im.plane[0]);
  const DG_GLOBAL uint8_t *pB = gp<const uint8_t>(im.plane[1]);
  const DG_GLOBAL uint8_t *pR = gp<const uint8_t>(im.plane[2]);
  const uint32_t sY = im.cbw[0] * 8, sC = im.cbw[1] * 8;
  FillRaw f;
  f.y = *(const DG_GLOBAL u32x2 *)(pY + (size_t)__umul24(y, sY) + x0);
  if (SS == 0) {
    f.b0 = *(const DG_GLOBAL u32x2 *)(pB + (size_t)__umul24(y, sC) + x0);
    f.r0 = *(const DG_GLOBAL u32x2 *)(pR + (size_t)__umul24(y, sC) + x0);
    f.b1 = f.r1 = u32x2{0, 0};
  } else {
    const uint32_t c0 = x0 >> 1;
    uint32_t rr = y, rn = y;
    if (SS == 2) {
      rr = y >> 1;
      const uint32_t last = Z ? im.cbh[1] * 8 - 1 : im.cdsh[1] - 1;
      rn = (y & 1) ? (rr + 1 <= last ? rr + 1 : last) : (rr > 0 ? rr - 1 : 0);
    }
    f.b0 = *(const DG_GLOBAL u32x2 *)(pB + (size_t)__umul24(rr, 2 * sC) + 2 * c0);
    f.r0 = *(const DG_GLOBAL u32x2 *)(pR + (size_t)__umul24(rr, 2 * sC) + 2 * c0);
    if (SS == 2) {
      f.b1 = *(const DG_GLOBAL u32x2 *)(pB + (size_t)__umul24(rn, 2 * sC) + 2 * c0);
      f.r1 = *(const DG_GLOBAL u32x2 *)(pR + (size_t)__umul24(rn, 2 * sC) + 2 * c0);
    } else {
      f.b1 = f.r1 = u32x2{0, 0};
    }
  }
  return f;
}

template <int FC>
__device__ __forceinline__ void hcolor_fc8(const ImageDesc &im, const FillRaw &f, uint32_t x0, uint32_t v[8]) {
  constexpr bool Z = FC == FC_420_Z || FC == FC_422_Z || FC == FC_444_Z;
  constexpr int SS = (FC == FC_420 || FC == FC_420_Z) ? 2 : (FC == FC_422 || FC == FC_422_Z) ? 1 : 0;
  int32_t Yv[8], Cb[8], Cr[8];
  auto unpack8 = [](u32x2 w, int32_t o[8]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      o[k] = (w.x >> (8 * k)) & 0xFF;
      o[k + 4] = (w.y >> (8 * k)) & 0xFF;
    }
  };
  auto rec6 = [](u32x2 w, int32_t cs[6]) {  // load_crec6's unpacking (dg_plane.h)
    cs[0] = (int32_t)(w.y & 0xFF);
#pragma unroll
    for (int k = 0; k < 4; k++) cs[k + 1] = (int32_t)((w.x >> (8 * k)) & 0xFF);
    cs[5] = (int32_t)((w.y >> 8) & 0xFF);
  };
  unpack8(f.y, Yv);
  if (SS == 0) {
    unpack8(f.b0, Cb);
    unpack8(f.r0, Cr);
  } else {
    const uint32_t sC = im.cbw[1] * 8, c0 = x0 >> 1;
    int32_t b[6], r[6];
    rec6(f.b0, b);
    rec6(f.r0, r);
    if (SS == 2) {
      int32_t b1[6], r1[6];
      rec6(f.b1, b1);
      rec6(f.r1, r1);
#pragma unroll
      for (int k = 0; k < 6; k++) {
        b[k] = Z ? (3 * b[k] + 2 + b1[k]) >> 2 : 3 * b[k] + b1[k];
        r[k] = Z ? (3 * r[k] + 2 + r1[k]) >> 2 : 3 * r[k] + r1[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (Z) {  // zune: (3a + b + 2) >> 2 both phases; the padded row's last pair is its quirk
        const int32_t ab = 3 * b[k + 1] + 2, ar = 3 * r[k + 1] + 2;
        int32_t eb = (ab + b[k]) >> 2, ob = (ab + b[k + 2]) >> 2, er = (ar + r[k]) >> 2, orr = (ar + r[k + 2]) >> 2;
        if (c0 + (uint32_t)k + 1 == sC) {
          eb = (3 * b[k] + b[k + 1] + 2) >> 2;
          ob = b[k + 1];
          er = (3 * r[k] + r[k + 1] + 2) >> 2;
          orr = r[k + 1];
        }
        Cb[2 * k] = eb;
        Cb[2 * k + 1] = ob;
        Cr[2 * k] = er;
        Cr[2 * k + 1] = orr;
      } else if (SS == 2) {  // libjpeg h2v2 fancy over column sums
        Cb[2 * k] = (b[k + 1] * 3 + b[k] + 8) >> 4;
        Cb[2 * k + 1] = (b[k + 1] * 3 + b[k + 2] + 7) >> 4;
        Cr[2 * k] = (r[k + 1] * 3 + r[k] + 8) >> 4;
        Cr[2 * k + 1] = (r[k + 1] * 3 + r[k + 2] + 7) >> 4;
      } else {  // libjpeg h2v1 fancy
        Cb[2 * k] = (b[k + 1] * 3 + b[k] + 1) >> 2;
        Cb[2 * k + 1] = (b[k + 1] * 3 + b[k + 2] + 2) >> 2;
        Cr[2 * k] = (r[k + 1] * 3 + r[k] + 1) >> 2;
        Cr[2 * k + 1] = (r[k + 1] * 3 + r[k + 2] + 2) >> 2;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint8_t rr, gg, bb;
    if (Z)
      ycc_to_rgb_zune(Yv[k], Cb[k], Cr[k], rr, gg, bb);
    else
      ycc_to_rgb(Yv[k], Cb[k], Cr[k], rr, gg, bb);
    v[k] = (uint32_t)rr | ((uint32_t)gg << 8) | ((uint32_t)bb << 16);
  }
}

// 8 fused-fill pixels (RGB in bytes 0..2 of v[k]) into the band's LDS
// segment, one dword per pixel.  (A layout of i16 pixel pairs per channel,
// the dot2 operands as they are, measured neutral in round 4 and was
// dropped: the convolution is not issue-bound.)
__device__ __forceinline__ void hput8(const uint32_t v[8], uint32_t *seg) {
  u32x4 *d4 = (u32x4 *)seg;
  d4[0] = u32x4{v[0], v[1], v[2], v[3]};
  d4[1] = u32x4{v[4], v[5], v[6], v[7]};
}

// 4 source pixels at p (p % 4 == 0) of an interleaved C-byte row of `in_size`
// pixels in rows of `stride` (multiple of 4) bytes
__device__ __forceinline__ void hfill_bytes4(const DG_GLOBAL uint8_t *row, uint32_t C, uint32_t stride,
                                             uint32_t in_size, uint32_t p, uint32_t *d) {
  uint32_t v[4] = {0, 0, 0, 0};
  if ((p + 4) * C <= stride) {
    const DG_GLOBAL uint32_t *s4 = (const DG_GLOBAL uint32_t *)(row + (size_t)p * C);
    if (C == 3) {
      const uint32_t w0 = s4[0], w1 = s4[1], w2 = s4[2];
      v[0] = w0 & 0xFFFFFFu;
      v[1] = (w0 >> 24) | ((w1 & 0xFFFFu) << 8);
      v[2] = (w1 >> 16) | ((w2 & 0xFFu) << 16);
      v[3] = w2 >> 8;
    } else if (C == 1) {
      const uint32_t w = s4[0];
      v[0] = w & 0xFF;
      v[1] = (w >> 8) & 0xFF;
      v[2] = (w >> 16) & 0xFF;
      v[3] = w >> 24;
    } else if (C == 4) {
      v[0] = s4[0];
      v[1] = s4[1];
      v[2] = s4[2];
      v[3] = s4[3];
    } else {  // C == 2
      const uint32_t w0 = s4[0], w1 = s4[1];
      v[0] = w0 & 0xFFFF;
      v[1] = w0 >> 16;
      v[2] = w1 & 0xFFFF;
      v[3] = w1 >> 16;
    }
  } else {
    for (uint32_t k = 0; k < 4; k++)
      if (p + k < in_size)
        for (uint32_t ch = 0; ch < C; ch++) v[k] |= (uint32_t)row[(size_t)(p + k) * C + ch] << (8 * ch);
  }
  *(u32x4 *)d = u32x4{v[0], v[1], v[2], v[3]};
}

typedef short s16x2 __attribute__((ext_vector_type(2)));

template <int KMAX, int C, uint32_t SEGSTRIDE = kHSegStride, bool RING = false>
__device__ __forceinline__ void hconv_rows(const uint32_t *seg, uint32_t off, const uint32_t *kw2,
                                           const DG_GLOBAL int16_t *kp, uint32_t ksize, uint32_t n, uint32_t r0,
                                           uint32_t nrows, int32_t prec, uint8_t *ob, uint32_t col,
                                           uint32_t *ring = nullptr, uint32_t ring_row0 = 0) {
  constexpr uint32_t R = kHBandRows / 2;  // rows r0, r0 + 2, ...
  const int32_t bias = 1 << (prec - 1);
  int32_t a[R][C];
#pragma unroll
  for (uint32_t r = 0; r < R; r++)
#pragma unroll
    for (int c = 0; c < C; c++) a[r][c] = bias;
  if (KMAX > 0) {
    // two taps per v_dot2_i32_i16: the channel-c bytes of pixels i and i+1
    // packed as i16 x 2 (one v_perm) against the packed weights (w_i, w_i+1);
    // an odd last tap pairs with a zero weight.  Integer sums: bit-exact
    // with tap-by-tap accumulation.  Pairs start at the even position at or
    // below the window start (kw2 carries a leading zero weight for odd
    // starts), so each pair is one 8-byte-aligned ds_read_b64: half the LDS
    // instructions, and banked over 64 dwords instead of 32, so the lanes'
    // stride-s reads (s = the downscale factor) stop conflicting up to s = 2.
    const uint32_t offe = off & ~1u;
#pragma unroll
    for (int j = 0; j < (KMAX > 0 ? (KMAX + 1) / 2 : 1); j++) {
      if ((uint32_t)(2 * j) >= ksize + 1) break;
      const s16x2 w = __builtin_bit_cast(s16x2, kw2[j]);
#pragma unroll
      for (uint32_t r = 0; r < R; r++) {
        const u32x2 vv = *(const u32x2 *)(seg + (r0 + 2 * r) * SEGSTRIDE + offe + 2 * j);
        const uint32_t v0 = vv.x, v1 = vv.y;
#pragma unroll
        for (int c = 0; c < C; c++) {
          const uint32_t sel = 0x0C000C00u | ((4u + (uint32_t)c) << 16) | (uint32_t)c;  // [v0.c, 0, v1.c, 0]
          const uint32_t pr = __builtin_amdgcn_perm(v1, v0, sel);
          a[r][c] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pr), w, a[r][c], false);
        }
      }
    }
  } else {
    for (uint32_t i = 0; i < n; i++) {
      const int32_t w = kp[i];
#pragma unroll
      for (uint32_t r = 0; r < R; r++) {
        const uint32_t v = seg[(r0 + 2 * r) * SEGSTRIDE + off + i];
#pragma unroll
        for (int c = 0; c < C; c++) a[r][c] += (int32_t)((v >> (8 * c)) & 0xFF) * w;
      }
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < R; r++)
    if (r0 + 2 * r < nrows) {
      if (RING) {  // one dword per pixel into row (ring_row0 + r0 + 2r) of the H+V kernel's ring
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < C; c++) v |= (uint32_t)clip_shift(a[r][c], prec) << (8 * c);
        ring[((ring_row0 + r0 + 2 * r) % kHVRing) * kHBandCols + col] = v;
      } else {
        uint8_t *o = ob + (r0 + 2 * r) * (kHBandCols * 4) + col * C;
#pragma unroll
        for (int c = 0; c < C; c++) o[c] = clip_shift(a[r][c], prec);
      }
    }
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
template <class T, class S>
__device__ __forceinline__ T bcast(S v) {
  return __builtin_bit_cast(T, v);
}

// One octet of a zune fill (hcolor_fc8<FC_4xx_Z>'s arithmetic; SS = 2
// 4:2:0, 1 4:2:2, 0 4:4:4) as u16 pairs per channel: R[i] = (pixel 2i,
// pixel 2i + 1) of the octet.
template <int SS>
__device__ __forceinline__ void hpl_zune(const ImageDesc &im, const FillRaw &f, uint32_t x0, uint32_t R[4],
                                         uint32_t G[4], uint32_t B[4]) {
  u16x2 Cp[2][4];  // Cb, Cr: pixel pairs (0,1), (2,3), (4,5), (6,7)
  if (SS == 0) {  // full-rate chroma: the plane bytes as they are
#pragma unroll
    for (int pl = 0; pl < 2; pl++) {
      const u32x2 w = pl ? f.r0 : f.b0;
#pragma unroll
      for (int i = 0; i < 4; i++)
        Cp[pl][i] = bcast<u16x2>(__builtin_amdgcn_perm(0u, i < 2 ? w.x : w.y, (i & 1) ? 0x0C030C02u : 0x0C010C00u));
    }
  } else {
    // the 6 samples of a chroma record (load_crec6's order: left neighbour,
    // 4 samples, right neighbour) as 3 pairs
    auto rec3 = [](u32x2 w, u16x2 c[3]) {
      c[0] = bcast<u16x2>(__builtin_amdgcn_perm(w.x, w.y, 0x0C040C00u));
      c[1] = bcast<u16x2>(__builtin_amdgcn_perm(0u, w.x, 0x0C020C01u));
      c[2] = bcast<u16x2>(__builtin_amdgcn_perm(w.y, w.x, 0x0C050C03u));
    };
    const bool edge = (x0 >> 1) + 4u == im.cbw[1] * 8u;  // the padded chroma row's last 4 samples: zune's quirk
    const u16x2 two = {2, 2}, three = {3, 3};
#pragma unroll
    for (int pl = 0; pl < 2; pl++) {
      u16x2 c[3];
      rec3(pl ? f.r0 : f.b0, c);
      if (SS == 2) {  // vertical: (3 near + far + 2) >> 2
        u16x2 fa[3];
        rec3(pl ? f.r1 : f.b1, fa);
#pragma unroll
        for (int i = 0; i < 3; i++) c[i] = (c[i] * three + fa[i] + two) >> 2;
      }
      // horizontal: even_k = (3 c[k+1] + 2 + c[k]) >> 2, odd_k = (3 c[k+1] + 2 + c[k+2]) >> 2
      const u16x2 s12 =
          bcast<u16x2>(__builtin_amdgcn_perm(bcast<uint32_t>(c[1]), bcast<uint32_t>(c[0]), 0x05040302u));
      const u16x2 s34 =
          bcast<u16x2>(__builtin_amdgcn_perm(bcast<uint32_t>(c[2]), bcast<uint32_t>(c[1]), 0x05040302u));
      const u16x2 t12 = s12 * three + two, t34 = s34 * three + two;
      const uint32_t e01 = bcast<uint32_t>((t12 + c[0]) >> 2), o01 = bcast<uint32_t>((t12 + c[1]) >> 2);
      uint32_t e23 = bcast<uint32_t>((t34 + c[1]) >> 2), o23 = bcast<uint32_t>((t34 + c[2]) >> 2);
      if (edge) {  // even_3 = (3 c[3] + c[4] + 2) >> 2 (= odd_2), odd_3 = c[4]
        e23 = __builtin_amdgcn_perm(o23, e23, 0x05040100u);
        o23 = __builtin_amdgcn_perm(bcast<uint32_t>(c[2]), o23, 0x05040100u);
      }
      Cp[pl][0] = bcast<u16x2>(__builtin_amdgcn_perm(o01, e01, 0x05040100u));
      Cp[pl][1] = bcast<u16x2>(__builtin_amdgcn_perm(o01, e01, 0x07060302u));
      Cp[pl][2] = bcast<u16x2>(__builtin_amdgcn_perm(o23, e23, 0x05040100u));
      Cp[pl][3] = bcast<u16x2>(__builtin_amdgcn_perm(o23, e23, 0x07060302u));
    }
  }
  const s16x2 c128 = {128, 128}, zero = {0, 0}, c255 = {255, 255};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t yw = i < 2 ? f.y.x : f.y.y;
    const s16x2 y = bcast<s16x2>(__builtin_amdgcn_perm(0u, yw, (i & 1) ? 0x0C030C02u : 0x0C010C00u));
    const s16x2 xcb = bcast<s16x2>(Cp[0][i]) - c128, xcr = bcast<s16x2>(Cp[1][i]) - c128;
    // ycc_to_rgb_zune in 16 bits: every product and sum fits (|x| <= 128)
    s16x2 r = y + ((xcr * (s16x2){45, 45}) >> 5);
    s16x2 g = y - ((xcb * (s16x2){11, 11} + xcr * (s16x2){23, 23}) >> 5);
    s16x2 b = y + ((xcb * (s16x2){113, 113}) >> 6);
    r = __builtin_elementwise_min(__builtin_elementwise_max(r, zero), c255);
    g = __builtin_elementwise_min(__builtin_elementwise_max(g, zero), c255);
    b = __builtin_elementwise_min(__builtin_elementwise_max(b, zero), c255);
    R[i] = bcast<uint32_t>(r);
    G[i] = bcast<uint32_t>(g);
    B[i] = bcast<uint32_t>(b);
  }
}

// u16 pairs per channel -> pixel dwords (RGB in bytes 0..2)
__device__ __forceinline__ void hpl_join(const uint32_t R[4], const uint32_t G[4], const uint32_t B[4], uint32_t v[8]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t rg = __builtin_amdgcn_perm(G[i], R[i], 0x06020400u);  // r0 g0 r1 g1
    v[2 * i] = __builtin_amdgcn_perm(B[i], rg, 0x0C040100u);
    v[2 * i + 1] = __builtin_amdgcn_perm(B[i], rg, 0x0C060302u);
  }
}

// pixel dwords (RGB in bytes 0..2) -> u16 pairs per channel
__device__ __forceinline__ void hpl_split(const uint32_t v[8], uint32_t R[4], uint32_t G[4], uint32_t B[4]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    R[i] = __builtin_amdgcn_perm(v[2 * i + 1], v[2 * i], 0x0C040C00u);
    G[i] = __builtin_amdgcn_perm(v[2 * i + 1], v[2 * i], 0x0C050C01u);
    B[i] = __builtin_amdgcn_perm(v[2 * i + 1], v[2 * i], 0x0C060C02u);
  }
}

// LDS source segment (pixels per row) of a band H kernel, per weight class:
// a window of <= 8 taps means a downscale of at most ~1.2x, <= 16 taps at most
// ~2.5x, so 128 output columns read at most 192 / 384 source pixels (the host
// promotes a pass to the next class when h_pass_span says otherwise).  The
// smaller segments let 8 workgroups share a CU instead of 6 (LDS-bound).
constexpr uint32_t hseg_px(int kmax) { return kmax == 8 ? 192u : kmax == 16 ? 384u : kHSegPx; }
constexpr uint32_t hpl_stride(int kmax) { return hseg_px(kmax) / 2 + 4; }  // dwords per row-channel plane

// FUSED: the first pass of a colour JPEG (fill = upsample + colour
// conversion from the planes, C = 3); otherwise the fill copies interleaved
// bytes of C = 1..4 channels.  Separate kernels so each allocates registers
// for its own path only.
template <int KMAX, bool FUSED, int FC = FC_GENERIC, bool PF = false>
__device__ __forceinline__ void hband(const ImageDesc &im, const ResizePass &ps, uint32_t item, uint32_t *seg,
                                      uint8_t *ob, uint32_t *ext) {
  constexpr uint32_t SEGPX = hseg_px(KMAX), SS = SEGPX + 8;  // pixels per row; row stride (dwords)
  // one workgroup: a tile of kHBandCols output columns x ps.bands bands of
  // kHBandRows rows; the column tile's weights, source extent and descriptor
  // reads are set up once and reused for every band
  const uint32_t tiles = (ps.width + kHBandCols - 1) / kHBandCols;
  const uint32_t group = item / tiles, tile = item - group * tiles;
  const uint32_t x0 = tile * kHBandCols;
  const uint32_t x1 = x0 + kHBandCols < ps.width ? x0 + kHBandCols : ps.width;
  // coefficient tables cover all out_size outputs; this pass computes [out0, out0 + width)
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;
  const uint32_t C = FUSED ? 3u : ps.C, ksize = ps.ksize;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ksize;
  const uint32_t t = threadIdx.x, col = t & (kHBandCols - 1), x = x0 + col;
  const bool valid = x < x1;
  // Source segment of the tile.  Trimmed window starts are not strictly
  // monotone (an exactly-zero edge weight is dropped), so take the min/max.
  uint32_t st = 0, n = 0;
  if (valid) {
    st = (uint32_t)bounds[2 * x];
    n = (uint32_t)bounds[2 * x + 1];
  }
  if (t == 0) {
    ext[0] = 0xFFFFFFFFu;
    ext[1] = 0;
  }
  __syncthreads();
  if (valid && t < kHBandCols) {
    atomicMin(&ext[0], st);
    atomicMax(&ext[1], st + ksize);
  }
  __syncthreads();
  const uint32_t p0 = ext[0] & ~7u;
  uint32_t p1 = ext[1];
  if (p1 - p0 > SEGPX) p1 = p0 + SEGPX;  // host sizing guarantees this never triggers
  const uint32_t pe = p1 < ps.in_size ? p1 : ps.in_size;
  uint32_t kw2[KMAX > 0 ? (KMAX + 1) / 2 : 1];  // weights (w_2j, w_2j+1) as i16 x 2
  const DG_GLOBAL int16_t *kp = coef + (size_t)(valid ? x : x0) * ksize;
  if (KMAX > 0) {
    // pair j covers segment positions offe + 2j, offe + 2j + 1 = taps 2j - sh, 2j + 1 - sh
    const uint32_t sh = (st - p0) & 1u;
#pragma unroll
    for (int j = 0; j < (KMAX > 0 ? (KMAX + 1) / 2 : 1); j++) {
      const int32_t tl = 2 * j - (int32_t)sh, th = tl + 1;
      const uint32_t lo = (valid && tl >= 0 && (uint32_t)tl < n) ? (uint16_t)kp[tl] : 0u;
      const uint32_t hi = (valid && (uint32_t)th < n) ? (uint16_t)kp[th] : 0u;
      kw2[j] = lo | (hi << 16);
    }
  }
  static_assert(kHBandRows * 32 == 256, "store mapping");
  const uint32_t fr = t >> 5, fl = t & 31;  // store: 32 threads per row
  const uint32_t off = st - p0, r0 = t / kHBandCols;
  // Fill jobs (an octet, or a 4-pixel unit, of one row) are numbered across
  // the band's rows, so all 256 threads share them and waves with no job
  // skip the fill: mapping 32 threads to each row left most lanes of the
  // last pass idle (a 2x downscale's 35 octets per row ran two full passes
  // for 3 octets), and every wave ran it.  Row of job j = j / per-row count
  // n, by a 24-bit multiply with ceil(2^20 / n): exact for every j < 8n and
  // n <= 160 (kHSegPx / 4 units; checked exhaustively), product < 2^32.
  const uint32_t njob_row = FUSED ? (pe - p0 + 7) >> 3 : (pe - p0 + 3) >> 2;
  const uint32_t inv_row = ((1u << 20) - 1u + njob_row) / (njob_row ? njob_row : 1u);
  const int32_t prec = ps.precision;
  const uint32_t rb = (x1 - x0) * C;  // <= kHBandCols * 4 = 512 bytes: 32 chunks of 16
  const uint32_t ybeg = group * kHBandRows * ps.bands;
  // specialised fused fills prefetch (option "h_prefetch", ImageDesc... pass mode kHPrefetch)
  constexpr bool PREFETCH = FUSED && FC != FC_GENERIC && PF;
  FillRaw pre;
  if (PREFETCH && ybeg < ps.rows) {  // band 0's first job
    const uint32_t nr0 = ps.rows - ybeg < kHBandRows ? ps.rows - ybeg : kHBandRows;
    if (t < nr0 * njob_row) {
      const uint32_t r = __umul24(t, inv_row) >> 20, q = t - r * njob_row;
      pre = hload_fc8<FC>(im, ps.row0 + ybeg + r, p0 + 8 * q);
    }
  }
  for (uint32_t bi = 0; bi < ps.bands; bi++) {
    const uint32_t y0 = ybeg + bi * kHBandRows;
    if (y0 >= ps.rows) break;
    const uint32_t nrows = ps.rows - y0 < kHBandRows ? ps.rows - y0 : kHBandRows;
    // phase 1: fill
    const uint32_t njob = nrows * njob_row;
    for (uint32_t j = t; j < njob; j += 256) {
      const uint32_t r = __umul24(j, inv_row) >> 20, q = j - r * njob_row;
      if (FUSED) {
        uint32_t v[8];
        if (FC == FC_GENERIC) {
          hcolor8(im, ps.row0 + y0 + r, p0 + 8 * q, v);
        } else {
          // a thread's first job of the band was loaded before the previous
          // band's convolution (pre); later ones load here
          const FillRaw f = (PREFETCH && j == t) ? pre : hload_fc8<FC>(im, ps.row0 + y0 + r, p0 + 8 * q);
          if (FC == FC_420_Z || FC == FC_422_Z || FC == FC_444_Z) {
            uint32_t Rw[4], Gw[4], Bw[4];  // the planar kernel's packed zune fill, back to pixel dwords
            hpl_zune<FC == FC_420_Z ? 2 : FC == FC_422_Z ? 1 : 0>(im, f, p0 + 8 * q, Rw, Gw, Bw);
            hpl_join(Rw, Gw, Bw, v);
          } else {
            hcolor_fc8<FC>(im, f, p0 + 8 * q, v);
          }
        }
        hput8(v, seg + r * SS + 8 * q);
      } else {
        const DG_GLOBAL uint8_t *src = gp<const uint8_t>(ps.src) + (size_t)(ps.row0 + y0 + r) * ps.src_stride;
        hfill_bytes4(src, C, ps.src_stride, ps.in_size, p0 + 4 * q, seg + r * SS + 4 * q);
      }
    }
    __syncthreads();
    if (PREFETCH) {  // the next band's first fill job: its loads overlap this band's convolution
      const uint32_t y1 = y0 + kHBandRows;
      if (bi + 1 < ps.bands && y1 < ps.rows) {
        const uint32_t nr1 = ps.rows - y1 < kHBandRows ? ps.rows - y1 : kHBandRows;
        if (t < nr1 * njob_row) {
          const uint32_t r = __umul24(t, inv_row) >> 20, q = t - r * njob_row;
          pre = hload_fc8<FC>(im, ps.row0 + y1 + r, p0 + 8 * q);
        }
      }
    }
    // phase 2: convolve (thread: column col, rows r0, r0 + 2, ...)
    if (valid) {
      if (FUSED || C == 3)
        hconv_rows<KMAX, 3, SS>(seg, off, kw2, kp, ksize, n, r0, nrows, prec, ob, col);
      else if (C == 1)
        hconv_rows<KMAX, 1, SS>(seg, off, kw2, kp, ksize, n, r0, nrows, prec, ob, col);
      else if (C == 4)
        hconv_rows<KMAX, 4, SS>(seg, off, kw2, kp, ksize, n, r0, nrows, prec, ob, col);
      else
        hconv_rows<KMAX, 2, SS>(seg, off, kw2, kp, ksize, n, r0, nrows, prec, ob, col);
    }
    __syncthreads();
    // phase 3: store the band's rows, 16 bytes per thread per step (the next
    // band's fill only touches seg; its barrier orders these ob reads before
    // the next convolution writes ob)
    DG_GLOBAL uint8_t *dst = gp<uint8_t>(ps.dst) + (size_t)y0 * ps.dst_stride + (size_t)x0 * C;
    if (fr < nrows && fl * 16 < rb) {
      const uint32_t r = fr, b = fl * 16;
      DG_GLOBAL uint8_t *d = dst + (size_t)r * ps.dst_stride + b;
      const uint8_t *o = ob + r * (kHBandCols * 4) + b;
      if (b + 16 <= rb && (((uintptr_t)d) & 15) == 0) {
        *(DG_GLOBAL u32x4 *)d = *(const u32x4 *)o;
      } else {
        const uint32_t e = b + 16 < rb ? 16 : rb - b;
        for (uint32_t i = 0; i < e; i++) d[i] = o[i];
      }
    }
  }
}

// Register budget for 5 waves per SIMD (<= 96 VGPRs; every variant fits
// without scratch: 64-95 VGPRs).  A 4-wave budget measured slower
// (resize_h1 2.81-2.90 vs 2.69-2.74 ms) and is no longer built.  The 8-tap
// kernels fit 6 waves (80 VGPRs, no scratch; their 10 KiB of LDS allows it);
// the 16-tap ones would spill at 6.
template <int KMAX, bool FUSED, bool PF = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KMAX == 8 ? 6 : 5))) void k_resize_hb(
    const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list, int stage) {
  __shared__ __attribute__((aligned(16))) uint32_t seg[kHBandRows * (hseg_px(KMAX) + 8)];
  __shared__ __attribute__((aligned(16))) uint8_t ob[kHBandRows * kHBandCols * 4];
  __shared__ uint32_t ext[2];
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  const ImageDesc &im = imgs[it.image];
  const ResizePass &ps = im.pass[stage];
  if (FUSED) {  // a fused fill reads the planes: specialised per layout (uniform per workgroup)
    switch (fill_class(im)) {
      case FC_420: hband<KMAX, FUSED, FC_420, PF>(im, ps, it.item0, seg, ob, ext); return;
      case FC_420_Z: hband<KMAX, FUSED, FC_420_Z, PF>(im, ps, it.item0, seg, ob, ext); return;
      case FC_422: hband<KMAX, FUSED, FC_422, PF>(im, ps, it.item0, seg, ob, ext); return;
      case FC_422_Z: hband<KMAX, FUSED, FC_422_Z, PF>(im, ps, it.item0, seg, ob, ext); return;
      case FC_444: hband<KMAX, FUSED, FC_444, PF>(im, ps, it.item0, seg, ob, ext); return;
      case FC_444_Z: hband<KMAX, FUSED, FC_444_Z, PF>(im, ps, it.item0, seg, ob, ext); return;
      default: break;
    }
  }
  hband<KMAX, FUSED, FC_GENERIC, false>(im, ps, it.item0, seg, ob, ext);
}

// ---- band H pass over a planar segment (option "h_planar", k_resize_hbp)
//
// The first pass of a colour JPEG with up to 16 taps, as k_resize_hb<K,
// true> computes it (same work items, fill jobs, weights and sums: the
// bytes are equal), but the band's LDS segment holds each row's channels
// as planes of u16 pixel pairs -- pixel 2i in the low half of dword i, 2i + 1
// in the high half, the v_dot2_i32_i16 operand as it is -- instead of one
// dword per pixel.  The convolution then reads one dword per tap pair and
// channel and feeds it to the dot2 unchanged (k_resize_hb spends a v_perm
// per tap pair and channel building that operand from pixel dwords), and
// the 4:2:0 zune fill (the configs[1] headline's layout) upsamples and
// colour-converts two pixels per instruction in packed 16-bit arithmetic,
// its results already in that layout (4:2:2 and 4:4:4 zune fills too).
// The libjpeg-mode and generic fills convert their pixel dwords (three
// v_perm per pixel pair).
//   A measured split of k_resize_hb<16> (round 6, resize_h1 1.80 ms per
// configs[1] batch): without the fill arithmetic 1.28 ms, without the
// convolution 1.24, without the plane loads 1.68 -- the kernel follows its
// VALU work, not its loads.
template <int KMAX, uint32_t SPS>
__device__ __forceinline__ void hconv_rows_pl(const uint32_t *segp, uint32_t pb, const uint32_t *kw2, uint32_t ksize,
                                              uint32_t r0, uint32_t nrows, int32_t prec, uint8_t *ob, uint32_t col) {
  constexpr uint32_t R = kHBandRows / 2;  // rows r0, r0 + 2, ...
  const int32_t bias = 1 << (prec - 1);
  int32_t a[R][3];
#pragma unroll
  for (uint32_t r = 0; r < R; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) a[r][c] = bias;
  // (Two pairs per step, their 24 reads issued together, measured slower:
  // resize_h1 1.69-1.72 vs 1.65-1.70 ms, round 6.)
#pragma unroll
  for (int j = 0; j < (KMAX + 1) / 2; j++) {
    if ((uint32_t)(2 * j) >= ksize + 1) break;
    const s16x2 w = bcast<s16x2>(kw2[j]);
#pragma unroll
    for (uint32_t r = 0; r < R; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const uint32_t pr = segp[((r0 + 2 * r) * 3 + c) * SPS + pb + j];
        a[r][c] = __builtin_amdgcn_sdot2(bcast<s16x2>(pr), w, a[r][c], false);
      }
  }
#pragma unroll
  for (uint32_t r = 0; r < R; r++)
    if (r0 + 2 * r < nrows) {
      uint8_t *o = ob + (r0 + 2 * r) * (kHBandCols * 4) + col * 3;
#pragma unroll
      for (int c = 0; c < 3; c++) o[c] = clip_shift(a[r][c], prec);
    }
}

template <int KMAX, int FC, bool PF>
__device__ __forceinline__ void hband_pl(const ImageDesc &im, const ResizePass &ps, uint32_t item, uint32_t *segp,
                                         uint8_t *ob, uint32_t *ext) {
  static_assert(KMAX == 8 || KMAX == 16, "planar segments for the 8- and 16-tap classes");
  constexpr uint32_t SEGPX = hseg_px(KMAX), SPS = hpl_stride(KMAX);
  const uint32_t tiles = (ps.width + kHBandCols - 1) / kHBandCols;
  const uint32_t group = item / tiles, tile = item - group * tiles;
  const uint32_t x0 = tile * kHBandCols;
  const uint32_t x1 = x0 + kHBandCols < ps.width ? x0 + kHBandCols : ps.width;
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;
  const uint32_t ksize = ps.ksize;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ksize;
  const uint32_t t = threadIdx.x, col = t & (kHBandCols - 1), x = x0 + col;
  const bool valid = x < x1;
  uint32_t st = 0, n = 0;
  if (valid) {
    st = (uint32_t)bounds[2 * x];
    n = (uint32_t)bounds[2 * x + 1];
  }
  if (t == 0) {
    ext[0] = 0xFFFFFFFFu;
    ext[1] = 0;
  }
  __syncthreads();
  if (valid && t < kHBandCols) {
    atomicMin(&ext[0], st);
    atomicMax(&ext[1], st + ksize);
  }
  __syncthreads();
  const uint32_t p0 = ext[0] & ~7u;
  uint32_t p1 = ext[1];
  if (p1 - p0 > SEGPX) p1 = p0 + SEGPX;  // host sizing guarantees this never triggers
  const uint32_t pe = p1 < ps.in_size ? p1 : ps.in_size;
  uint32_t kw2[(KMAX + 1) / 2];  // weights (w_2j, w_2j+1) as i16 x 2
  const DG_GLOBAL int16_t *kp = coef + (size_t)(valid ? x : x0) * ksize;
  {
    const uint32_t sh = (st - p0) & 1u;
#pragma unroll
    for (int j = 0; j < (KMAX + 1) / 2; j++) {
      const int32_t tl = 2 * j - (int32_t)sh, th = tl + 1;
      const uint32_t lo = (valid && tl >= 0 && (uint32_t)tl < n) ? (uint16_t)kp[tl] : 0u;
      const uint32_t hi = (valid && (uint32_t)th < n) ? (uint16_t)kp[th] : 0u;
      kw2[j] = lo | (hi << 16);
    }
  }
  const uint32_t fr = t >> 5, fl = t & 31;  // store: 32 threads per row
  const uint32_t pb = (st - p0) >> 1, r0 = t / kHBandCols;  // pair index of the window's first pair
  const uint32_t njob_row = (pe - p0 + 7) >> 3;
  const uint32_t inv_row = ((1u << 20) - 1u + njob_row) / (njob_row ? njob_row : 1u);
  const int32_t prec = ps.precision;
  const uint32_t rb = (x1 - x0) * 3;
  const uint32_t ybeg = group * kHBandRows * ps.bands;
  constexpr bool PREFETCH = FC != FC_GENERIC && PF;
  FillRaw pre;
  if (PREFETCH && ybeg < ps.rows) {
    const uint32_t nr0 = ps.rows - ybeg < kHBandRows ? ps.rows - ybeg : kHBandRows;
    if (t < nr0 * njob_row) {
      const uint32_t r = __umul24(t, inv_row) >> 20, q = t - r * njob_row;
      pre = hload_fc8<FC>(im, ps.row0 + ybeg + r, p0 + 8 * q);
    }
  }
  for (uint32_t bi = 0; bi < ps.bands; bi++) {
    const uint32_t y0 = ybeg + bi * kHBandRows;
    if (y0 >= ps.rows) break;
    const uint32_t nrows = ps.rows - y0 < kHBandRows ? ps.rows - y0 : kHBandRows;
    const uint32_t njob = nrows * njob_row;
    for (uint32_t j = t; j < njob; j += 256) {
      const uint32_t r = __umul24(j, inv_row) >> 20, q = j - r * njob_row;
      uint32_t Rw[4], Gw[4], Bw[4];
      if (FC == FC_GENERIC) {
        uint32_t v[8];
        hcolor8(im, ps.row0 + y0 + r, p0 + 8 * q, v);
        hpl_split(v, Rw, Gw, Bw);
      } else {
        const FillRaw f = (PREFETCH && j == t) ? pre : hload_fc8<FC>(im, ps.row0 + y0 + r, p0 + 8 * q);
        if (FC == FC_420_Z || FC == FC_422_Z || FC == FC_444_Z) {
          hpl_zune<FC == FC_420_Z ? 2 : FC == FC_422_Z ? 1 : 0>(im, f, p0 + 8 * q, Rw, Gw, Bw);
        } else {
          uint32_t v[8];
          hcolor_fc8<FC>(im, f, p0 + 8 * q, v);
          hpl_split(v, Rw, Gw, Bw);
        }
      }
      uint32_t *d = segp + r * 3 * SPS + 4 * q;
      *(u32x4 *)d = u32x4{Rw[0], Rw[1], Rw[2], Rw[3]};
      *(u32x4 *)(d + SPS) = u32x4{Gw[0], Gw[1], Gw[2], Gw[3]};
      *(u32x4 *)(d + 2 * SPS) = u32x4{Bw[0], Bw[1], Bw[2], Bw[3]};
    }
    __syncthreads();
    if (PREFETCH) {
      const uint32_t y1 = y0 + kHBandRows;
      if (bi + 1 < ps.bands && y1 < ps.rows) {
        const uint32_t nr1 = ps.rows - y1 < kHBandRows ? ps.rows - y1 : kHBandRows;
        if (t < nr1 * njob_row) {
          const uint32_t r = __umul24(t, inv_row) >> 20, q = t - r * njob_row;
          pre = hload_fc8<FC>(im, ps.row0 + y1 + r, p0 + 8 * q);
        }
      }
    }
    if (valid) hconv_rows_pl<KMAX, SPS>(segp, pb, kw2, ksize, r0, nrows, prec, ob, col);
    __syncthreads();
    DG_GLOBAL uint8_t *dst = gp<uint8_t>(ps.dst) + (size_t)y0 * ps.dst_stride + (size_t)x0 * 3;
    if (fr < nrows && fl * 16 < rb) {
      const uint32_t r = fr, b = fl * 16;
      DG_GLOBAL uint8_t *d = dst + (size_t)r * ps.dst_stride + b;
      const uint8_t *o = ob + r * (kHBandCols * 4) + b;
      if (b + 16 <= rb && (((uintptr_t)d) & 15) == 0) {
        *(DG_GLOBAL u32x4 *)d = *(const u32x4 *)o;
      } else {
        const uint32_t e = b + 16 < rb ? 16 : rb - b;
        for (uint32_t i = 0; i < e; i++) d[i] = o[i];
      }
    }
  }
}

// Z: the zune fill classes (the drop-in's decode semantics), else the
// libjpeg ones; an image of the other semantics in the batch takes the
// generic fill (bit-exact, slower).  Split so that each kernel holds only its
// own fills' registers: the zune 16-tap kernel fits 6 waves per SIMD (80
// VGPRs; its zune paths spill nothing -- only the rare generic fill reloads a
// few words per band), +2% headline over 5 waves (round 6); the libjpeg one
// keeps 5.  8 taps: 6 waves, without the next-band prefetch (which would
// spill there; measured level with it).
template <int KMAX, bool PF, bool Z>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KMAX == 8 || Z ? 6 : 5))) void k_resize_hbp(
    const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list, int stage) {
  __shared__ __attribute__((aligned(16))) uint32_t segp[kHBandRows * 3 * hpl_stride(KMAX)];
  __shared__ __attribute__((aligned(16))) uint8_t ob[kHBandRows * kHBandCols * 4];
  __shared__ uint32_t ext[2];
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  const ImageDesc &im = imgs[it.image];
  const ResizePass &ps = im.pass[stage];
  const int fc = fill_class(im);
  if (Z) {
    switch (fc) {
      case FC_420_Z: hband_pl<KMAX, FC_420_Z, PF>(im, ps, it.item0, segp, ob, ext); return;
      case FC_422_Z: hband_pl<KMAX, FC_422_Z, PF>(im, ps, it.item0, segp, ob, ext); return;
      case FC_444_Z: hband_pl<KMAX, FC_444_Z, PF>(im, ps, it.item0, segp, ob, ext); return;
      default: break;
    }
  } else {
    switch (fc) {
      case FC_420: hband_pl<KMAX, FC_420, PF>(im, ps, it.item0, segp, ob, ext); return;
      case FC_422: hband_pl<KMAX, FC_422, PF>(im, ps, it.item0, segp, ob, ext); return;
      case FC_444: hband_pl<KMAX, FC_444, PF>(im, ps, it.item0, segp, ob, ext); return;
      default: break;
    }
  }
  hband_pl<KMAX, FC_GENERIC, false>(im, ps, it.item0, segp, ob, ext);
}

// ---- band H pass on the matrix cores (k_resize_hm)
//
// Same work items as k_resize_hb (kHBandCols output columns x 8 * ps.bands
// rows), in bands of 16 rows.  The fill stages the band's source segment in
// LDS as planar signed bytes (p - 128), one plane per channel; the
// convolution out[row][x] = sum_k src[row][k] * w_x[k] of a 16-column
// subtile is the product of a banded K x 16 weight matrix with the 16 x K
// band, v_mfma_i32_16x16x64_i8 over the subtile's window (KS steps of 64).
// The i16 weight splits into three i8 digits, w = 2^14 a + 2^7 b + c (a in
// [-2, 1], b and c in [0, 127]: fast_image_resize's precision puts the
// largest weight of a pass in [2^14, 2^15)), the pixel offset comes back as
// 128 * sum(w) in the accumulator's initial value: every product and sum is
// an exact i32, so the bytes equal the VALU kernel's (and the oracle's) bit
// for bit.  A = the weight digits (output column n = lane & 15, K group
// g = lane >> 4), B = the pixels (band row n, K group g), so lane (n, g)
// receives output columns 4g..4g+3 of band row n -- 4 adjacent pixels,
// stored straight to HBM (C x 4 bytes) without an LDS staging pass.
typedef int i32x4m __attribute__((ext_vector_type(4)));
constexpr uint32_t kHmRows = 16;                      // band rows = MFMA M
// planar rows: reads reach 64 * KS past a subtile's 16-aligned window start;
// an odd multiple of 16 bytes keeps the 16 rows of a lane group on distinct banks
constexpr uint32_t hm_row_stride(uint32_t need) {
  uint32_t a = (need + 15) / 16 * 16;
  while (((a / 16) & 1u) == 0) a += 16;
  return a;
}

template <int KS, bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_resize_hm(
    const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list, int stage) {
  constexpr uint32_t AS = hm_row_stride(kHSegPx + 64 * KS);
  constexpr uint32_t NP = FUSED ? 3 : 4;  // planes (channels)
  __shared__ __attribute__((aligned(16))) uint8_t ap[NP * kHmRows * AS];
  __shared__ __attribute__((aligned(16))) int32_t corr[kHBandCols];
  __shared__ uint32_t ext[2];
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  const ImageDesc &im = imgs[it.image];
  const ResizePass &ps = im.pass[stage];
  const uint32_t tiles = (ps.width + kHBandCols - 1) / kHBandCols;
  const uint32_t group = it.item0 / tiles, tile = it.item0 - group * tiles;
  const uint32_t x0 = tile * kHBandCols;
  const uint32_t x1 = x0 + kHBandCols < ps.width ? x0 + kHBandCols : ps.width;
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;
  const uint32_t C = FUSED ? 3u : ps.C, ksize = ps.ksize;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ksize;
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
  if (t == 0) {
    ext[0] = 0xFFFFFFFFu;
    ext[1] = 0;
  }
  __syncthreads();
  if (t < kHBandCols && x0 + t < x1) {
    const uint32_t st = (uint32_t)bounds[2 * (x0 + t)], n = (uint32_t)bounds[2 * (x0 + t) + 1];
    atomicMin(&ext[0], st);
    atomicMax(&ext[1], st + n);
  }
  __syncthreads();
  const uint32_t p0 = ext[0] & ~15u;  // 16-aligned: the B operand reads are 16-byte LDS reads
  const uint32_t pe = ext[1] < ps.in_size ? ext[1] : ps.in_size;
  const int32_t prec = ps.precision;

  // weights of this wave's two subtiles (2 * wave, 2 * wave + 1), set up once
  const uint32_t n = lane & 15, g = lane >> 4;
  i32x4m wlo[2][KS], wmd[2][KS], whi[2][KS];
  uint32_t k0[2], steps[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t sub = wave * 2 + j;
    const uint32_t xs = x0 + sub * 16 + n;
    const bool valid = xs < x1;
    uint32_t st = 0, cnt = 0;
    if (valid) {
      st = (uint32_t)bounds[2 * xs];
      cnt = (uint32_t)bounds[2 * xs + 1];
    }
    uint32_t mn = valid ? st : 0xFFFFFFFFu, mx = valid ? st + cnt : 0u;
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      const uint32_t a = (uint32_t)__shfl_xor((int)mn, m, 64), b = (uint32_t)__shfl_xor((int)mx, m, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    k0[j] = mn == 0xFFFFFFFFu ? p0 : (mn & ~15u);
    steps[j] = mx > k0[j] ? (mx - k0[j] + 63) / 64 : 0;
    if (steps[j] > (uint32_t)KS) steps[j] = KS;  // the host sends windows <= 64 * KS (h_mfma_class)
    const DG_GLOBAL int16_t *kp = coef + (size_t)(valid ? xs : x0) * ksize;
    int32_t sum = 0;  // of column n's weights: this lane's K groups, then over the four groups
#pragma unroll
    for (int s = 0; s < KS; s++) {
      uint32_t lo[4] = {0, 0, 0, 0}, md[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
      const int32_t kb = (int32_t)(k0[j] + 64 * s + 16 * g) - (int32_t)st;
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int32_t i = kb + e;
        const int32_t w = (valid && i >= 0 && i < (int32_t)cnt) ? (int32_t)kp[i] : 0;
        sum += w;
        lo[e >> 2] |= (uint32_t)(w & 127) << (8 * (e & 3));
        md[e >> 2] |= (uint32_t)((w >> 7) & 127) << (8 * (e & 3));
        hi[e >> 2] |= (uint32_t)((w >> 14) & 0xFF) << (8 * (e & 3));
      }
      wlo[j][s] = i32x4m{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]};
      wmd[j][s] = i32x4m{(int)md[0], (int)md[1], (int)md[2], (int)md[3]};
      whi[j][s] = i32x4m{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if (g == 0) corr[sub * 16 + n] = sum * 128 + (1 << (prec - 1));
  }
  // fill jobs (an octet of one row, or a 4-pixel unit) numbered across the band's rows
  const uint32_t njob_row = FUSED ? (pe - p0 + 7) >> 3 : (pe - p0 + 3) >> 2;
  const uint32_t inv_row = ((1u << 20) - 1u + njob_row) / (njob_row ? njob_row : 1u);
  const uint32_t ybeg = group * kHBandRows * ps.bands, yend0 = ybeg + kHBandRows * ps.bands;
  const uint32_t yend = yend0 < ps.rows ? yend0 : ps.rows;
  __syncthreads();
  for (uint32_t y0 = ybeg; y0 < yend; y0 += kHmRows) {
    const uint32_t nrows = yend - y0 < kHmRows ? yend - y0 : kHmRows;
    // phase 1: fill (rows past nrows keep stale bytes: their outputs are not stored)
    const uint32_t njob = nrows * njob_row;
    for (uint32_t j = t; j < njob; j += 256) {
      const uint32_t r = __umul24(j, inv_row) >> 20, q = j - r * njob_row;
      if (FUSED) {
        int32_t Y[8], Cb[8], Cr[8];
        upsample_ycc8(im, p0 + 8 * q, ps.row0 + y0 + r, Y, Cb, Cr);
        uint32_t R[2] = {0, 0}, G[2] = {0, 0}, B[2] = {0, 0};
#pragma unroll
        for (int k = 0; k < 8; k++) {
          uint8_t rr, gg, bb;
          ycc_px(im, Y[k], Cb[k], Cr[k], rr, gg, bb);
          R[k >> 2] |= (uint32_t)rr << (8 * (k & 3));
          G[k >> 2] |= (uint32_t)gg << (8 * (k & 3));
          B[k >> 2] |= (uint32_t)bb << (8 * (k & 3));
        }
        uint8_t *d = ap + r * AS + 8 * q;
        *(u32x2 *)d = u32x2{R[0] ^ 0x80808080u, R[1] ^ 0x80808080u};
        *(u32x2 *)(d + kHmRows * AS) = u32x2{G[0] ^ 0x80808080u, G[1] ^ 0x80808080u};
        *(u32x2 *)(d + 2 * kHmRows * AS) = u32x2{B[0] ^ 0x80808080u, B[1] ^ 0x80808080u};
      } else {
        uint32_t v[4];
        const DG_GLOBAL uint8_t *src = gp<const uint8_t>(ps.src) + (size_t)(ps.row0 + y0 + r) * ps.src_stride;
        hfill_bytes4(src, C, ps.src_stride, ps.in_size, p0 + 4 * q, v);
        uint8_t *d = ap + r * AS + 4 * q;
        for (uint32_t c = 0; c < C; c++) {
          const uint32_t sh = 8 * c;
          const uint32_t w = ((v[0] >> sh) & 0xFFu) | (((v[1] >> sh) & 0xFFu) << 8) | (((v[2] >> sh) & 0xFFu) << 16) |
                             (((v[3] >> sh) & 0xFFu) << 24);
          *(uint32_t *)(d + c * kHmRows * AS) = w ^ 0x80808080u;
        }
      }
    }
    __syncthreads();
    // phase 2: convolve on the matrix cores, store 4 pixels per lane
    const uint32_t yr = y0 + n;  // this lane's output row
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t sub = wave * 2 + j;
      if (x0 + sub * 16 >= x1 || steps[j] == 0) continue;  // wave-uniform
      uint32_t px[4] = {0, 0, 0, 0};  // channel c of columns 4g .. 4g+3
      for (uint32_t c = 0; c < C; c++) {
        const uint8_t *brow = ap + c * kHmRows * AS + n * AS + (k0[j] - p0) + 16 * g;
        i32x4m alo = *(const i32x4m *)(corr + sub * 16 + 4 * g), amd = {0, 0, 0, 0}, ahi = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < KS; s++) {
          if (s > 0 && steps[j] <= (uint32_t)s) break;
          const i32x4m b = *(const i32x4m *)(brow + 64 * s);
          alo = __builtin_amdgcn_mfma_i32_16x16x64_i8(wlo[j][s], b, alo, 0, 0, 0);
          amd = __builtin_amdgcn_mfma_i32_16x16x64_i8(wmd[j][s], b, amd, 0, 0, 0);
          ahi = __builtin_amdgcn_mfma_i32_16x16x64_i8(whi[j][s], b, ahi, 0, 0, 0);
        }
        uint32_t o[4];
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
          const int32_t v = ((ahi[rr] << 14) + (amd[rr] << 7) + alo[rr]) >> prec;
          o[rr] = (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
        const uint32_t w4 = pack4(o[0], o[1], o[2], o[3]);
        px[0] = c == 0 ? w4 : px[0];
        px[1] = c == 1 ? w4 : px[1];
        px[2] = c == 2 ? w4 : px[2];
        px[3] = c == 3 ? w4 : px[3];
      }
      const uint32_t xs = x0 + sub * 16 + 4 * g;  // the lane's first column
      if (n >= nrows || xs >= x1) continue;
      DG_GLOBAL uint8_t *d = gp<uint8_t>(ps.dst) + (size_t)yr * ps.dst_stride + (size_t)xs * C;
      // interleave the channels of the 4 pixels: C x 4 bytes
      uint32_t w[4] = {0, 0, 0, 0};
      if (C == 1) {
        w[0] = px[0];
      } else if (C == 2) {
        w[0] = __builtin_amdgcn_perm(px[1], px[0], 0x05010400u);  // L0 A0 L1 A1
        w[1] = __builtin_amdgcn_perm(px[1], px[0], 0x07030602u);  // L2 A2 L3 A3
      } else if (C == 3) {
        const uint32_t rg = __builtin_amdgcn_perm(px[1], px[0], 0x05010400u);   // R0 G0 R1 G1
        const uint32_t rg2 = __builtin_amdgcn_perm(px[1], px[0], 0x07030602u);  // R2 G2 R3 G3
        w[0] = __builtin_amdgcn_perm(px[2], rg, 0x02040100u);                   // R0 G0 B0 R1
        const uint32_t gb = __builtin_amdgcn_perm(px[2], rg, 0x0c0c0503u);      // G1 B1 0 0
        w[1] = __builtin_amdgcn_perm(rg2, gb, 0x05040100u);                     // G1 B1 R2 G2
        w[2] = __builtin_amdgcn_perm(rg2, px[2], 0x03070602u);                  // B2 R3 G3 B3
      } else {
        const uint32_t rg = __builtin_amdgcn_perm(px[1], px[0], 0x05010400u);   // R0 G0 R1 G1
        const uint32_t rg2 = __builtin_amdgcn_perm(px[1], px[0], 0x07030602u);  // R2 G2 R3 G3
        const uint32_t ba = __builtin_amdgcn_perm(px[3], px[2], 0x05010400u);   // B0 A0 B1 A1
        const uint32_t ba2 = __builtin_amdgcn_perm(px[3], px[2], 0x07030602u);  // B2 A2 B3 A3
        w[0] = __builtin_amdgcn_perm(ba, rg, 0x05040100u);                      // R0 G0 B0 A0
        w[1] = __builtin_amdgcn_perm(ba, rg, 0x07060302u);                      // R1 G1 B1 A1
        w[2] = __builtin_amdgcn_perm(ba2, rg2, 0x05040100u);
        w[3] = __builtin_amdgcn_perm(ba2, rg2, 0x07060302u);
      }
      if (xs + 4 <= x1 && (((uintptr_t)d) & 3) == 0) {
        DG_GLOBAL uint32_t *d4 = (DG_GLOBAL uint32_t *)d;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          if (k < C) d4[k] = w[k];
      } else {
        const uint32_t nb = (x1 - xs < 4 ? x1 - xs : 4) * C;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++)
          if (k < nb) d[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
      }
    }
    __syncthreads();  // the next band's fill overwrites the planes
  }
}

// Fused first H + V pass of a colour JPEG (ImageDesc pass[0] mode kHVFused):
// one workgroup = kHBandCols columns x kHVRows V output rows.  It computes
// the H rows those outputs' windows span, band by band exactly as
// k_resize_hb does (fill from the Y/Cb/Cr planes, same weights and sums),
// keeps them in an LDS ring, and after each band produces every V row whose
// window is complete (two rows at a time: thread = column x row parity; tap
// pairs by v_dot2 as k_resize_v).  The H intermediate (about 1.1 GB per
// configs[1] batch) never reaches HBM; rows at segment borders are computed
// by both neighbours.  Integer sums: bit-exact with the two-pass path.
template <int KMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_resize_hv(
    const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  __shared__ __attribute__((aligned(16))) uint32_t seg[kHBandRows * kHVSegStride];
  __shared__ __attribute__((aligned(16))) uint32_t ring[kHVRing * kHBandCols];
  __shared__ __attribute__((aligned(16))) uint8_t ob[kHVOut * kHBandCols * 3];
  __shared__ uint32_t ext[4];
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  const ImageDesc &im = imgs[it.image];
  const ResizePass &ps = im.pass[0], &pv = im.pass[1];
  const uint32_t tiles = (ps.width + kHBandCols - 1) / kHBandCols;
  const uint32_t sg = it.item0 / tiles, tile = it.item0 - sg * tiles;
  const uint32_t x0 = tile * kHBandCols;
  const uint32_t x1 = x0 + kHBandCols < ps.width ? x0 + kHBandCols : ps.width;
  const uint32_t oy0 = sg * kHVRows, oy1 = oy0 + kHVRows < pv.rows ? oy0 + kHVRows : pv.rows;
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;
  const DG_GLOBAL int32_t *vb = gp<const int32_t>(pv.bounds) + 2 * pv.out0;
  const uint32_t ksize = ps.ksize;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ksize;
  const uint32_t t = threadIdx.x, col = t & (kHBandCols - 1), x = x0 + col;
  const bool valid = x < x1;
  uint32_t st = 0, n = 0;
  if (valid) {
    st = (uint32_t)bounds[2 * x];
    n = (uint32_t)bounds[2 * x + 1];
  }
  if (t == 0) {
    ext[0] = 0xFFFFFFFFu;
    ext[1] = 0;
    ext[2] = 0xFFFFFFFFu;
    ext[3] = 0;
  }
  __syncthreads();
  if (valid && t < kHBandCols) {
    atomicMin(&ext[0], st);
    atomicMax(&ext[1], st + ksize);
  }
  if (t < oy1 - oy0) {  // the H rows the segment's V windows span (starts are not strictly monotone)
    const int32_t vs = vb[2 * (oy0 + t)], vn = vb[2 * (oy0 + t) + 1];
    atomicMin(&ext[2], (uint32_t)vs);
    atomicMax(&ext[3], (uint32_t)(vs + vn));
  }
  __syncthreads();
  const uint32_t p0 = __builtin_amdgcn_readfirstlane(ext[0]) & ~7u;
  uint32_t p1 = __builtin_amdgcn_readfirstlane(ext[1]);
  if (p1 - p0 > kHVSegPx) p1 = p0 + kHVSegPx;  // host sizing guarantees this never triggers
  const uint32_t pe = p1 < ps.in_size ? p1 : ps.in_size;
  const uint32_t hy0 = __builtin_amdgcn_readfirstlane(ext[2]), hy1 = __builtin_amdgcn_readfirstlane(ext[3]);
  uint32_t kw2[KMAX > 0 ? (KMAX + 1) / 2 : 1];
  const DG_GLOBAL int16_t *kp = coef + (size_t)(valid ? x : x0) * ksize;
  {
    const uint32_t sh = (st - p0) & 1u;
#pragma unroll
    for (int j = 0; j < (KMAX + 1) / 2; j++) {
      const int32_t tl = 2 * j - (int32_t)sh, th = tl + 1;
      const uint32_t lo = (valid && tl >= 0 && (uint32_t)tl < n) ? (uint16_t)kp[tl] : 0u;
      const uint32_t hi = (valid && (uint32_t)th < n) ? (uint16_t)kp[th] : 0u;
      kw2[j] = lo | (hi << 16);
    }
  }
  const uint32_t off = st - p0, r0 = t / kHBandCols;
  const uint32_t njob_row = (pe - p0 + 7) >> 3;
  const uint32_t inv_row = ((1u << 20) - 1u + njob_row) / (njob_row ? njob_row : 1u);
  const int32_t prec = ps.precision, vprec = pv.precision, vbias = 1 << (vprec - 1);
  const uint32_t vk = pv.ksize;
  const DG_GLOBAL int16_t *vcoef = gp<const int16_t>(pv.coef) + (size_t)pv.out0 * vk;
  const uint32_t rb = (x1 - x0) * 3;  // V output bytes per row of the tile (<= 384)
  uint32_t oy = oy0;
  for (uint32_t y0 = hy0; y0 < hy1; y0 += kHBandRows) {
    const uint32_t nrows = hy1 - y0 < kHBandRows ? hy1 - y0 : kHBandRows;
    // H: fill, convolve into the ring (rows y0 .. y0 + nrows - 1)
    const uint32_t njob = nrows * njob_row;
    for (uint32_t j = t; j < njob; j += 256) {
      const uint32_t r = __umul24(j, inv_row) >> 20, q = j - r * njob_row;
      hfill_color8(im, ps.row0 + y0 + r, p0 + 8 * q, seg + r * kHVSegStride + 8 * q);
    }
    __syncthreads();
    if (valid) hconv_rows<KMAX, 3, kHVSegStride, true>(seg, off, kw2, kp, ksize, n, r0, nrows, prec, nullptr, col,
                                                      ring, y0);
    __syncthreads();
    // V: every output row whose window is now complete, up to kHVOut per round
    // (thread = column x row parity, rows h, h + 2, ...)
    const uint32_t done = y0 + nrows;
    for (;;) {
      uint32_t nr = 0;
      while (nr < kHVOut && oy + nr < oy1 && (uint32_t)(vb[2 * (oy + nr)] + vb[2 * (oy + nr) + 1]) <= done) nr++;
      if (!nr) break;
      if (valid) {
        // h is wave-uniform (two waves per row parity): bounds and weights by scalar loads
        for (uint32_t h = __builtin_amdgcn_readfirstlane(t >> 7); h < nr; h += 2) {
          const uint32_t y = oy + h;
          const int32_t vs = vb[2 * y], vn = vb[2 * y + 1];
          const DG_GLOBAL int16_t *kv = vcoef + (size_t)y * vk;
          int32_t acc[3] = {vbias, vbias, vbias};
          int32_t i = 0;
          for (; i + 1 < vn; i += 2) {
            const uint32_t w2 = (uint32_t)(uint16_t)kv[i] | ((uint32_t)(uint16_t)kv[i + 1] << 16);
            const s16x2 w = __builtin_bit_cast(s16x2, w2);
            const uint32_t a0 = ring[((uint32_t)(vs + i) % kHVRing) * kHBandCols + col];
            const uint32_t a1 = ring[((uint32_t)(vs + i + 1) % kHVRing) * kHBandCols + col];
#pragma unroll
            for (int b = 0; b < 3; b++) {
              const uint32_t sel = 0x0C000C00u | ((4u + (uint32_t)b) << 16) | (uint32_t)b;  // [a0.b, 0, a1.b, 0]
              acc[b] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, __builtin_amdgcn_perm(a1, a0, sel)), w,
                                              acc[b], false);
            }
          }
          if (i < vn) {
            const int32_t w = kv[i];
            const uint32_t a0 = ring[((uint32_t)(vs + i) % kHVRing) * kHBandCols + col];
#pragma unroll
            for (int b = 0; b < 3; b++) acc[b] += (int32_t)((a0 >> (8 * b)) & 0xFF) * w;
          }
          uint8_t *o = ob + h * (kHBandCols * 3) + col * 3;
#pragma unroll
          for (int b = 0; b < 3; b++) o[b] = clip_shift(acc[b], vprec);
        }
      }
      __syncthreads();
      {  // store the rows: 16 bytes per thread, 24 threads per row (rb <= 384)
        for (uint32_t j = t; j < nr * 24; j += 256) {
          const uint32_t fr = j / 24, fl = j - fr * 24;
          if (fl * 16 >= rb) continue;
          DG_GLOBAL uint8_t *d = gp<uint8_t>(pv.dst) + (size_t)(oy + fr) * pv.dst_stride + (size_t)x0 * 3 + fl * 16;
          const uint8_t *src = ob + fr * (kHBandCols * 3) + fl * 16;
          if (fl * 16 + 16 <= rb && (((uintptr_t)d) & 15) == 0) {
            *(DG_GLOBAL u32x4 *)d = *(const u32x4 *)src;
          } else {
            const uint32_t e = fl * 16 + 16 <= rb ? 16 : rb - fl * 16;
            for (uint32_t i = 0; i < e; i++) d[i] = src[i];
          }
        }
      }
      __syncthreads();
      oy += nr;
    }
  }
}


// Vertical pass: each thread produces 16 consecutive bytes of one output row
// (channel-agnostic), one 16-byte load per tap: a wave streams 1 KiB of a
// source row per tap.
__global__ __launch_bounds__(256) void k_resize_v(const ImageDesc *__restrict__ imgs,
                                                  const WgItem *__restrict__ list, int stage) {
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  // stage in bits 0-7; bits 8+: consecutive 256-unit strides per workgroup
  // item (option "v_units"; the host lists one item per v_units * 256 units)
  const uint32_t vunits = (uint32_t)stage >> 8;
  const ResizePass &ps = imgs[it.image].pass[stage & 0xFF];
  const uint32_t rowbytes = ps.width * ps.C;
  const uint32_t units = (rowbytes + 15) / 16;
  for (uint32_t kv = 0; kv < vunits; kv++) {
  const uint32_t idx = it.item0 + kv * 256 + threadIdx.x;
  if (idx >= units * ps.rows) return;
  const uint32_t y = idx / units, u = idx - y * units;
  const uint32_t b0 = u * 16;
  const uint32_t nb = rowbytes - b0 < 16 ? rowbytes - b0 : 16;
  const uint32_t yc = y + ps.out0;  // coefficient row: the pass may compute a window of out_size
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds);
  const int32_t start = bounds[2 * yc], n = bounds[2 * yc + 1];
  const DG_GLOBAL int16_t *k = gp<const int16_t>(ps.coef) + (size_t)yc * ps.ksize;
  const int32_t prec = ps.precision, bias = 1 << (prec - 1);
  int32_t a[16];
#pragma unroll
  for (int j = 0; j < 16; j++) a[j] = bias;
  const DG_GLOBAL uint8_t *src = gp<const uint8_t>(ps.src) + (size_t)(start - (int32_t)ps.row0) * ps.src_stride + b0;
  if (nb == 16 && (ps.src_stride & 15) == 0) {
    // two taps (source rows i, i+1) per v_dot2_i32_i16, as in hconv_rows
    int32_t i = 0;
    for (; i + 1 < n; i += 2) {
      const uint32_t w2 = (uint32_t)(uint16_t)k[i] | ((uint32_t)(uint16_t)k[i + 1] << 16);
      const s16x2 w = __builtin_bit_cast(s16x2, w2);
      const u32x4 v0 = *(const DG_GLOBAL u32x4 *)(src + (size_t)i * ps.src_stride);
      const u32x4 v1 = *(const DG_GLOBAL u32x4 *)(src + (size_t)(i + 1) * ps.src_stride);
#pragma unroll
      for (int j = 0; j < 4; j++) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t sel = 0x0C000C00u | ((4u + (uint32_t)b) << 16) | (uint32_t)b;  // [v0.b, 0, v1.b, 0]
          const uint32_t pr = __builtin_amdgcn_perm(v1[j], v0[j], sel);
          a[4 * j + b] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pr), w, a[4 * j + b], false);
        }
      }
    }
    if (i < n) {
      const int32_t w = k[i];
      const u32x4 v = *(const DG_GLOBAL u32x4 *)(src + (size_t)i * ps.src_stride);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t x = v[j];
        a[4 * j] += (int32_t)(x & 0xFF) * w;
        a[4 * j + 1] += (int32_t)((x >> 8) & 0xFF) * w;
        a[4 * j + 2] += (int32_t)((x >> 16) & 0xFF) * w;
        a[4 * j + 3] += (int32_t)(x >> 24) * w;
      }
    }
  } else {
    for (int32_t i = 0; i < n; i++) {
      const int32_t w = k[i];
      const DG_GLOBAL uint8_t *sr = src + (size_t)i * ps.src_stride;
#pragma unroll
      for (int j = 0; j < 16; j++)
        if ((uint32_t)j < nb) a[j] += (int32_t)sr[j] * w;
    }
  }
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; j++)
    o[j] = pack4(clip_shift(a[4 * j], prec), clip_shift(a[4 * j + 1], prec), clip_shift(a[4 * j + 2], prec),
                 clip_shift(a[4 * j + 3], prec));
  DG_GLOBAL uint8_t *dst = gp<uint8_t>(ps.dst) + (size_t)y * ps.dst_stride + b0;
  if (nb == 16 && (ps.dst_stride & 15) == 0) {
    *(DG_GLOBAL u32x4 *)dst = u32x4{o[0], o[1], o[2], o[3]};
  } else if (nb == 16 && (ps.dst_stride & 3) == 0) {
    DG_GLOBAL uint32_t *d = (DG_GLOBAL uint32_t *)dst;
    d[0] = o[0];
    d[1] = o[1];
    d[2] = o[2];
    d[3] = o[3];
  } else {
    for (uint32_t j = 0; j < nb; j++) dst[j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
  }
  }
}

// Vertical pass on column tiles (option "v_tile" = R).
// One wave owns R consecutive output rows x 64 16-byte units (1 KiB) of one
// pass and walks the source rows their windows span once, in pairs: each
// source row is loaded once per tile instead of once per output row that
// uses it (k_resize_v re-loads all n taps for every output row and left the
// overlap to L2), and the byte-pair perms of a source-row pair are shared by
// the R outputs.  The R x pairs weight table (two i16 taps per dword, zero
// outside an output's window) is built per wave in LDS, in windows of
// kVtWCap / R pairs; a pair whose weights are both zero for an output is a
// scalar branch (the rows are wave-uniform).  Same arithmetic as k_resize_v
// (bias, v_dot2_i32_i16 over (row i, row i + 1) pairs, clip_shift), so the
// bytes are identical: a tap pair's zero weight adds exactly 0.
constexpr uint32_t kVtWCap = 256;  // packed weight pairs per wave in LDS

// 5 waves per SIMD for R <= 4: the prefetched pair needs 98 VGPRs
// unconstrained at R = 4 (4 waves: measured slower than without the
// prefetch); at 96 the compiler keeps one dword of setup in scratch, outside
// the row loop.  R = 8 (option value, not the default) is left unconstrained.
template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R <= 4 ? 5 : 1))) void k_resize_vt(const ImageDesc *__restrict__ imgs,
                                                   const WgItem *__restrict__ list, int stage) {
  __shared__ uint32_t wtab[4][kVtWCap];
  const WgItem it = list[xcd_remap(blockIdx.x, gridDim.x)];
  const ResizePass &ps = imgs[it.image].pass[stage];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t rowbytes = ps.width * ps.C;
  const uint32_t units = (rowbytes + 15) / 16;
  const uint32_t chunks = (units + 63) / 64;
  const uint32_t groups = (ps.rows + R - 1) / R;
  const uint32_t w = it.item0 + wv;  // this wave's tile
  if (w >= chunks * groups) return;  // (wave-uniform)
  const uint32_t g = w / chunks, c = w - g * chunks;
  const uint32_t y0 = g * R;
  const uint32_t nr = ps.rows - y0 < (uint32_t)R ? ps.rows - y0 : (uint32_t)R;
  const uint32_t u = c * 64 + lane;
  const uint32_t b0 = (u < units ? u : units - 1) * 16;  // lanes past the row load a valid unit, store nothing
  const uint32_t yc0 = y0 + ps.out0;                      // coefficient row of output row y0
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds);
  const DG_GLOBAL int16_t *kbase = gp<const int16_t>(ps.coef);
  const int32_t prec = ps.precision, bias = 1 << (prec - 1);
  // the span of source rows the tile's windows cover
  int32_t lo = 0x7FFFFFFF, hi = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    if ((uint32_t)r < nr) {
      const int32_t s = bounds[2 * (yc0 + r)], n = bounds[2 * (yc0 + r) + 1];
      lo = s < lo ? s : lo;
      hi = s + n > hi ? s + n : hi;
    }
  }
  const uint32_t npair = (uint32_t)(hi - lo + 1) >> 1;
  const uint32_t pwin = kVtWCap / R;  // pairs per weight-table window
  int32_t a[R][16];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int j = 0; j < 16; j++) a[r][j] = bias;
  const size_t sstride = ps.src_stride;
  const DG_GLOBAL uint8_t *src = gp<const uint8_t>(ps.src) + (size_t)(lo - (int32_t)ps.row0) * sstride + b0;
  uint32_t *wt = wtab[wv];
  for (uint32_t p0 = 0; p0 < npair; p0 += pwin) {
    const uint32_t pn = npair - p0 < pwin ? npair - p0 : pwin;
    __builtin_amdgcn_wave_barrier();  // the previous window's reads are issued (one wave: LDS in order)
    for (uint32_t e = lane; e < (uint32_t)R * pn; e += 64) {
      const uint32_t r = e / pn, p = e - r * pn;
      uint32_t pk = 0;
      if (r < nr) {
        const int32_t s = bounds[2 * (yc0 + r)], n = bounds[2 * (yc0 + r) + 1];
        const int32_t j = lo + 2 * (int32_t)(p0 + p) - s;  // tap index of the pair's first row
        const DG_GLOBAL int16_t *k = kbase + (size_t)(yc0 + r) * ps.ksize;
        const uint32_t w0 = (j >= 0 && j < n) ? (uint32_t)(uint16_t)k[j] : 0u;
        const uint32_t w1 = (j + 1 >= 0 && j + 1 < n) ? (uint32_t)(uint16_t)k[j + 1] : 0u;
        pk = w0 | (w1 << 16);
      }
      wt[r * pn + p] = pk;
    }
    __builtin_amdgcn_wave_barrier();
    // the next pair's rows are loaded while this pair's dot2s run: one
    // memory round trip per weight window instead of one per source-row pair
    // (resize_v1 0.57 -> 0.535 ms per configs[1] batch, round 6)
    auto ld = [&](uint32_t i, u32x4 &v0, u32x4 &v1) {
      v0 = *(const DG_GLOBAL u32x4 *)(src + (size_t)i * sstride);
      v1 = (int32_t)i + 1 < hi - lo ? *(const DG_GLOBAL u32x4 *)(src + (size_t)(i + 1) * sstride) : u32x4{0u, 0u, 0u, 0u};
    };
    u32x4 n0, n1;
    ld(2 * p0, n0, n1);
    for (uint32_t p = 0; p < pn; p++) {
      const uint32_t i = 2 * (p0 + p);  // source row lo + i (and lo + i + 1)
      const u32x4 v0 = n0, v1 = n1;
      uint32_t pr[16];
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int b = 0; b < 4; b++)
          pr[4 * j + b] = __builtin_amdgcn_perm(v1[j], v0[j], 0x0C000C00u | ((4u + (uint32_t)b) << 16) | (uint32_t)b);
      if (p + 1 < pn) ld(i + 2, n0, n1);
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t wp = __builtin_amdgcn_readfirstlane(wt[r * pn + p]);
        if (wp == 0u) continue;  // both taps outside output r's window (scalar branch)
        const s16x2 wv2 = __builtin_bit_cast(s16x2, wp);
#pragma unroll
        for (int q = 0; q < 16; q++) a[r][q] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pr[q]), wv2, a[r][q], false);
      }
    }
  }
  if (u >= units) return;
  const uint32_t nb = rowbytes - u * 16 < 16 ? rowbytes - u * 16 : 16;
#pragma unroll
  for (int r = 0; r < R; r++) {
    if ((uint32_t)r >= nr) break;
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
      o[j] = pack4(clip_shift(a[r][4 * j], prec), clip_shift(a[r][4 * j + 1], prec), clip_shift(a[r][4 * j + 2], prec),
                   clip_shift(a[r][4 * j + 3], prec));
    DG_GLOBAL uint8_t *dst = gp<uint8_t>(ps.dst) + (size_t)(y0 + r) * ps.dst_stride + u * 16;
    if (nb == 16 && (ps.dst_stride & 15) == 0) {
      *(DG_GLOBAL u32x4 *)dst = u32x4{o[0], o[1], o[2], o[3]};
    } else if (nb == 16 && (ps.dst_stride & 3) == 0) {
      DG_GLOBAL uint32_t *d = (DG_GLOBAL uint32_t *)dst;
      d[0] = o[0];
      d[1] = o[1];
      d[2] = o[2];
      d[3] = o[3];
    } else {
      for (uint32_t j = 0; j < nb; j++) dst[j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
    }
  }
}

// image 0.25 Rgba<u8>::blend of `f` over an opaque (128,128,128,255) pixel,
// then its RGB: f32 arithmetic in the crate's order, truncating casts.
// hipcc's f32 division is IEEE correctly rounded and contraction is off, so
// this matches the CPU restatement (oracle/png_oracle.c) bit for bit.
__device__ __forceinline__ void blend_over_gray(const DG_GLOBAL uint8_t *f, DG_GLOBAL uint8_t *o) {
  const uint32_t a = f[3];
  if (a == 0) {
    o[0] = o[1] = o[2] = 128;
    return;
  }
  if (a == 255) {
    o[0] = f[0];
    o[1] = f[1];
    o[2] = f[2];
    return;
  }
  const float mx = 255.0f;
  const float bg = 128.0f / mx, bga = 255.0f / mx;
  const float fa = (float)a / mx;
  const float af = bga + fa - bga * fa;
  if (af == 0.0f) {
    o[0] = o[1] = o[2] = 128;
    return;
  }
  const float bgm = bg * bga;
  for (int c = 0; c < 3; c++) {
    const float fc = (float)f[c] / mx;
    const float v = (fc * fa + bgm * (1.0f - fa)) / af;
    const float sv = mx * v;
    o[c] = (uint8_t)(sv < 0.0f ? 0 : sv > 255.0f ? 255 : (int)sv);
  }
}

__global__ __launch_bounds__(256) void k_copy(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const uint32_t idx = it.item0 + threadIdx.x;
  if (idx >= im.out_w * im.out_h) return;
  const uint32_t y = idx / im.out_w, x = idx - y * im.out_w;
  const DG_GLOBAL uint8_t *s = gp<const uint8_t>(im.final_src) + (size_t)y * im.final_src_stride + (size_t)x * im.final_src_c;
  DG_GLOBAL uint8_t *d = gp<uint8_t>(im.out) + (size_t)y * im.out_stride + (size_t)x * im.out_c;
  switch (im.copy_mode) {
    case 0:
      for (uint32_t c = 0; c < im.out_c; c++) d[c] = s[c];
      break;
    case 1:  // L8 -> RGB8 (image::DynamicImage::to_rgb8 replicates luma)
    case 4:  // unresized LumaA8 -> RGB8: alpha dropped
      d[0] = d[1] = d[2] = s[0];
      break;
    case 2:  // RGBA8 -> RGB8: Pixel::blend over opaque (128,128,128) (image_processing.rs:172-179)
      blend_over_gray(s, d);
      break;
    default: {  // resized LA: image_to_dyn_image made a GrayImage over the LA bytes
      const uint32_t rb = im.out_w * 2, r = idx / rb, c = idx - r * rb;
      const uint8_t v = gp<const uint8_t>(im.final_src)[(size_t)r * im.final_src_stride + c];
      d[0] = d[1] = d[2] = v;
      break;
    }
  }
}

// ------------------------------------------------------------ launchers

// Descriptor/list upload pulled by the GPU: 16-byte loads from the slot's
// page-locked staging buffer (mapped into the device's address space) into
// HBM.  hipMemcpyAsync of the ~2 MB meta region cost ~0.8 ms of the submitting
// thread's CPU per configs[1] batch (profiles/r04: host phase "h2d"), for a
// copy the GPU finishes in tens of microseconds.
__global__ __launch_bounds__(256) void k_meta_pull(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                   uint32_t n16) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

#define DG_LAUNCH(kern, nwg, st, ...)                                              \
  do {                                                                            \
    if (nwg) hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), 0, st, __VA_ARGS__); \
  } while (0)

void launch_destuff_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_destuff_count, nwg, st, imgs, list);
}
void launch_destuff_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_destuff_scan, nwg, st, imgs, list);
}
void launch_destuff_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_destuff_write, nwg, st, imgs, list);
}
void launch_destuff_one(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, uint64_t *state) {
  DG_LAUNCH(k_destuff_one, nwg, st, imgs, list, state);
}
// sync / fix hold only the batch's largest table count in LDS (4 for a
// typical colour JPEG instead of kMaxSlots = 6): 16 KiB instead of 23 KiB
// per workgroup, 8 resident workgroups per CU instead of 6
void launch_huff_sync(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                      const HuffTable *pool, SubState *subs, Ckpt *ck, BatchFlags *flags, bool stage,
                      uint32_t max_slots, uint32_t max_ac, bool pair, bool two) {
  if (!nwg) return;
  const size_t lds = (size_t)max_slots * sizeof(HuffTable) + ((size_t)max_ac << kMultiBits) * 2;
  const uint32_t multi = (max_ac ? 1u : 0u) | (pair ? 2u : 0u);  // bit 0: multi-symbol lookups, bit 1: pair steps
  if (two && !stage && !pair)  // two chains per lane (k_huff_sync2: no staging, no pair steps)
    hipLaunchKernelGGL(k_huff_sync2, dim3(nwg), dim3(128), lds, st, imgs, list, pool, subs, ck, flags, multi);
  else if (stage)
    hipLaunchKernelGGL(k_huff_sync<true>, dim3(nwg), dim3(256), lds, st, imgs, list, pool, subs, ck, flags, multi);
  else
    hipLaunchKernelGGL(k_huff_sync<false>, dim3(nwg), dim3(256), lds, st, imgs, list, pool, subs, ck, flags, multi);
}
void launch_huff_fix(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                     const HuffTable *pool, SubState *subs, Ckpt *ck, BatchFlags *flags, bool stage,
                     uint32_t max_slots) {
  if (!nwg) return;
  const size_t lds = (size_t)max_slots * sizeof(HuffTable);
  if (stage)
    hipLaunchKernelGGL(k_huff_fix<true>, dim3(nwg), dim3(256), lds, st, imgs, list, pool, subs, ck, flags);
  else
    hipLaunchKernelGGL(k_huff_fix<false>, dim3(nwg), dim3(256), lds, st, imgs, list, pool, subs, ck, flags);
}
void launch_huff_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, SubState *subs) {
  DG_LAUNCH(k_huff_scan, nwg, st, imgs, list, subs);
}
void launch_huff_write(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                       const HuffTable *pool, const SubState *subs, BatchFlags *flags, uint32_t max_slots,
                       const QuantTable *qpool, uint32_t pair, const Ckpt *ckpt) {
  if (!nwg) return;
  hipLaunchKernelGGL(k_huff_write, dim3(nwg), dim3(256), (size_t)max_slots * sizeof(HuffTable), st, imgs, list,
                     pool, subs, flags, qpool, pair, ckpt);
}
void launch_idct_list(hipStream_t st, const ImageDesc *imgs, const QuantTable *qpool, const BatchFlags *flags,
                      uint32_t nwg) {
  if (!nwg) return;
  DG_LAUNCH(k_idct_list, nwg, st, imgs, qpool, flags);
}
void launch_huff_scatter(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                         const SubState *subs) {
  DG_LAUNCH(k_huff_scatter, nwg, st, imgs, list, subs);
}
void launch_idct_t(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, const QuantTable *qpool) {
  if (nwg) hipLaunchKernelGGL(k_idct_t, dim3(nwg), dim3(64), 0, st, imgs, list, qpool);
}
void launch_idct(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, const QuantTable *qpool) {
  DG_LAUNCH(k_idct, nwg, st, imgs, list, qpool);
}
void launch_color(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_color, nwg, st, imgs, list);
}
void launch_coeffs(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_coeffs, nwg, st, imgs, list);
}
void launch_resize_h(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage) {
  DG_LAUNCH(k_resize_h, nwg, st, imgs, list, stage);
}
template <bool FUSED, bool PF = false>
static void launch_hb_classes(hipStream_t st, const ImageDesc *imgs, const WgItem *&list, const uint32_t ncls[4],
                              int stage) {
  DG_LAUNCH((k_resize_hb<8, FUSED, PF>), ncls[0], st, imgs, list, stage);
  list += ncls[0];
  DG_LAUNCH((k_resize_hb<16, FUSED, PF>), ncls[1], st, imgs, list, stage);
  list += ncls[1];
  DG_LAUNCH((k_resize_hb<32, FUSED, PF>), ncls[2], st, imgs, list, stage);
  list += ncls[2];
  DG_LAUNCH((k_resize_hb<0, FUSED>), ncls[3], st, imgs, list, stage);
  list += ncls[3];
}
// The fused classes with a planar segment (h_planar): 8 and 16 taps on
// k_resize_hbp, the wider ones on k_resize_hb (a planar 32-tap class, 35 KiB
// of LDS: 4 workgroups per CU instead of 5, measured level -- resize_h1
// 1.60-1.63 vs 1.62-1.64 ms, round 6 -- and was not kept)
template <bool PF, bool Z>
static void launch_hb_fused_planar(hipStream_t st, const ImageDesc *imgs, const WgItem *&list, const uint32_t ncls[4],
                                   int stage) {
  DG_LAUNCH((k_resize_hbp<8, false, Z>), ncls[0], st, imgs, list, stage);
  list += ncls[0];
  DG_LAUNCH((k_resize_hbp<16, PF, Z>), ncls[1], st, imgs, list, stage);
  list += ncls[1];
  DG_LAUNCH((k_resize_hb<32, true, PF>), ncls[2], st, imgs, list, stage);
  list += ncls[2];
  DG_LAUNCH((k_resize_hb<0, true>), ncls[3], st, imgs, list, stage);
  list += ncls[3];
}
void launch_resize_hb(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2][4],
                      int stage, bool prefetch, bool planar, bool zune) {
  if (planar && zune)
    prefetch ? launch_hb_fused_planar<true, true>(st, imgs, list, ncls[1], stage)
             : launch_hb_fused_planar<false, true>(st, imgs, list, ncls[1], stage);
  else if (planar)
    prefetch ? launch_hb_fused_planar<true, false>(st, imgs, list, ncls[1], stage)
             : launch_hb_fused_planar<false, false>(st, imgs, list, ncls[1], stage);
  else if (prefetch)
    launch_hb_classes<true, true>(st, imgs, list, ncls[1], stage);
  else
    launch_hb_classes<true, false>(st, imgs, list, ncls[1], stage);
  launch_hb_classes<false>(st, imgs, list, ncls[0], stage);
}
void launch_resize_hm(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2][2],
                      int stage) {
  DG_LAUNCH((k_resize_hm<1, true>), ncls[1][0], st, imgs, list, stage);
  list += ncls[1][0];
  DG_LAUNCH((k_resize_hm<2, true>), ncls[1][1], st, imgs, list, stage);
  list += ncls[1][1];
  DG_LAUNCH((k_resize_hm<1, false>), ncls[0][0], st, imgs, list, stage);
  list += ncls[0][0];
  DG_LAUNCH((k_resize_hm<2, false>), ncls[0][1], st, imgs, list, stage);
}
void launch_resize_hv(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2]) {
  DG_LAUNCH(k_resize_hv<8>, ncls[0], st, imgs, list);
  DG_LAUNCH(k_resize_hv<16>, ncls[1], st, imgs, list + ncls[0]);
}
void launch_resize_v(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage,
                     uint32_t vunits) {
  DG_LAUNCH(k_resize_v, nwg, st, imgs, list, stage | (int)(vunits << 8));
}
void launch_resize_vt(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage,
                      uint32_t rows) {
  if (rows == 8)
    DG_LAUNCH(k_resize_vt<8>, nwg, st, imgs, list, stage);
  else if (rows == 2)
    DG_LAUNCH(k_resize_vt<2>, nwg, st, imgs, list, stage);
  else
    DG_LAUNCH(k_resize_vt<4>, nwg, st, imgs, list, stage);
}
void launch_copy(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  DG_LAUNCH(k_copy, nwg, st, imgs, list);
}

void launch_meta_pull(hipStream_t st, const void *src, void *dst, size_t bytes) {
  const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
  const uint32_t nwg = (n16 + 255) / 256 < 1024u ? (n16 + 255) / 256 : 1024u;
  DG_LAUNCH(k_meta_pull, nwg, st, (const u32x4 *)src, (u32x4 *)dst, n16);
}

}  // namespace dg
