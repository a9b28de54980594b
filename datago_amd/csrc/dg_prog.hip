// dg_prog.hip — progressive JPEG entropy decoding on the GPU.
//
//   k_prog_zero   zero the coefficient blocks of progressive images
//   k_prog_scan   decode whole scans, one wave per scan, straight from the
//                 stuffed bytes (one launch per dependency level)
//
// What they restate: the progressive half of the reference's JPEG decode
// (zune-jpeg 0.5.12 "baseline + progressive", behind
// image 0.25.9 at worker_files.rs:8-17 / worker_wds.rs:45), written from T.81
// G.1.2 with libjpeg's jdphuff.c semantics, which oracle/jpeg_oracle.c
// restates on the CPU and the tests pin against PIL/libjpeg-turbo:
//   DC first    Huffman-coded DC difference, predictor per component, << Al
//   DC refine   one raw bit per block ORed in at bit Al
//   AC first    run/size symbols over the band [Ss, Se] of one component,
//               EOB runs (EOBn) spanning blocks, values << Al
//   AC refine   new +-1<<Al coefficients interleaved with correction bits
//               for the band's already-nonzero coefficients, EOB runs
// The coefficients land in the same MCU-interleaved, zigzag-ordered int16
// blocks the sequential decoder writes, so k_idct and everything after it
// are shared with the baseline path.
//
// Why one (wave-uniform) decoder per scan: a refinement scan's bit consumption depends on the
// coefficient history of the block it is in, so a decoder started at a
// guessed bit position cannot self-synchronise the way the sequential
// kernels (k_huff_sync) do; the scans of one file that touch disjoint
// (component, band) sets still run side by side (levels, see ProgScan).
#include <hip/hip_runtime.h>

#include "dg_entropy.h"
#include "dg_types.h"
#include "kernels.h"

namespace dg {

// ------------------------------------------------------------ zero

__global__ __launch_bounds__(256) void k_prog_zero(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  const uint64_t bytes = (uint64_t)im.total_blocks * 128;
  const uint64_t b0 = (uint64_t)it.item0 * kProgZeroBytes;
  const uint64_t b1 = b0 + kProgZeroBytes < bytes ? b0 + kProgZeroBytes : bytes;
  DG_GLOBAL u32x4 *p = (DG_GLOBAL u32x4 *)(gp<uint8_t>(im.coef) + b0);
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (uint64_t i = threadIdx.x; i * 16 < b1 - b0; i += 256) p[i] = z;  // blocks are 128 B: 16 B units
}

// ------------------------------------------------------------ wave-uniform scan decoder
//
// One 64-lane wave per scan.  The entropy decode is a serial chain, so every
// lane runs the same decode on the same state (uniform control flow, LDS
// reads are broadcasts) and the 64 lanes are spent on what is parallel:
// staging the stuffed stream into a 4 KiB LDS window with 16-byte loads,
// loading the Huffman tables, and moving coefficient blocks between HBM and
// LDS 64 at a time (only the scan's band [Ss, Se] is written back, so scans
// of other bands of the same blocks may run at the same time).  The decode
// itself then touches only LDS and registers.
constexpr uint32_t kPWin = 4096;  // stuffed-stream window (bytes)
constexpr uint32_t kPBlk = 64;    // coefficient blocks per chunk

struct ProgSmem {
  HuffTable tabs[4];
  int16_t blk[kPBlk][64];
  uint64_t nzm[kPBlk];  // refine scans: nonzero-history mask of each staged block (bit k = zigzag k)
  uint64_t cor[kPBlk];  //   correction bits in stream order (one per history-nonzero band position)
  uint32_t ncor[kPBlk]; //   how many
  uint64_t nwp[kPBlk];  //   new coefficients +1 << Al
  uint64_t nwn[kPBlk];  //   new coefficients -1 << Al
  uint8_t win[kPWin + 16];
};

// Every lane runs the same decode: make that explicit, so the state lives in
// SGPRs and the decode runs on the scalar unit (LDS reads return VGPRs).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

struct WReader {
  uint64_t d;       // absolute address of the scan's first byte
  uint32_t len;     // scan bytes
  uint32_t p;       // next byte to consume (relative to d)
  uint64_t wabs;    // absolute address of win[0] (16-byte aligned)
  uint64_t buf;     // MSB-first bit window
  int32_t nbits;
  uint32_t marker;  // a marker was reached: zeros are fed (libjpeg jpeg_fill_bit_buffer)
};

// window starting at the 16-byte line holding byte p; all 64 lanes load
__device__ __forceinline__ void wr_refill(WReader &r, ProgSmem &sm, uint32_t p) {
  __syncthreads();
  r.wabs = (r.d + p) & ~(uint64_t)15;
  const uint64_t end = r.d + r.len;
  constexpr uint32_t kPer = kPWin / 16 / 64;  // 16-byte lines per lane
  u32x4 v[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; i++) {  // all loads in flight before the LDS writes
    const uint64_t a = r.wabs + (uint64_t)(threadIdx.x + 64 * i) * 16;
    v[i] = a < end ? *(const DG_GLOBAL u32x4 *)(uintptr_t)a : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (uint32_t i = 0; i < kPer; i++) *(u32x4 *)&sm.win[(threadIdx.x + 64 * i) * 16] = v[i];
  __syncthreads();
}

// byte q (< len) of the scan, refilling the window when q is past it
__device__ __forceinline__ uint32_t wr_byte(WReader &r, ProgSmem &sm, uint32_t q) {
  if (r.d + q - r.wabs >= kPWin) wr_refill(r, sm, q);
  return uni(sm.win[r.d + q - r.wabs]);
}

__device__ __forceinline__ void wr_fill(WReader &r, ProgSmem &sm) {
  while (r.nbits <= 56) {
    // fast path: four bytes without an FF, inside the scan and the window
    if (!r.marker && r.nbits <= 32 && r.p + 4 <= r.len) {
      uint32_t idx = (uint32_t)(r.d + r.p - r.wabs);
      if (idx + 8 > kPWin) {
        wr_refill(r, sm, r.p);
        idx = (uint32_t)(r.d + r.p - r.wabs);
      }
      const uint32_t *w32 = (const uint32_t *)sm.win;
      const uint32_t lo = w32[idx >> 2], hi = w32[(idx >> 2) + 1];
      const uint32_t w = uni(__builtin_amdgcn_alignbyte(hi, lo, idx & 3));  // bytes p..p+3, little-endian
      if ((((~w) - 0x01010101u) & w & 0x80808080u) == 0) {             // no 0xFF byte
        r.buf |= (uint64_t)__builtin_bswap32(w) << (32 - r.nbits);
        r.nbits += 32;
        r.p += 4;
        continue;
      }
    }
    uint32_t c = 0;
    if (!r.marker && r.p < r.len) {
      c = wr_byte(r, sm, r.p);
      if (c == 0xFF) {
        uint32_t q = r.p + 1;
        while (q < r.len && wr_byte(r, sm, q) == 0xFF) q++;
        if (q < r.len && wr_byte(r, sm, q) == 0x00) {
          r.p = q + 1;
        } else {
          r.marker = 1;
          c = 0;
        }
      } else {
        r.p++;
      }
    }
    r.buf |= (uint64_t)c << (56 - r.nbits);
    r.nbits += 8;
  }
}

__device__ __forceinline__ uint32_t wr_get(WReader &r, ProgSmem &sm, uint32_t k) {
  if (k == 0) return 0;
  if (r.nbits < (int32_t)k) wr_fill(r, sm);
  const uint32_t v = (uint32_t)(r.buf >> (64 - k));
  r.buf <<= k;
  r.nbits -= (int32_t)k;
  return v;
}

// huff_lookup (dg_entropy.h) with uniform results
__device__ __forceinline__ uint32_t prog_lookup(const HuffTable &t, uint32_t bits) {
  const uint32_t e = uni(t.lut[bits >> (32 - kLutBits)]);
  if (!(e & 0x8000u) && e) return e;
  if (e & 0x8000u) {
    const uint32_t e2 = uni(t.sub[e & (kMaxSubTables - 1)][(bits >> (32 - 16)) & ((1u << kSubBits) - 1)]);
    return e2 ? e2 : (16u << 8);
  }
  const uint32_t pk = bits >> 16;
  for (int32_t l = kLutBits + 1; l <= 16; l++)
    if (pk < uni(t.lim[l])) return ((uint32_t)l << 8) | uni(t.vals[(uni((uint32_t)t.valoff[l]) + (pk >> (16 - l))) & 255]);
  return 16u << 8;
}

__device__ __forceinline__ uint32_t wr_sym(WReader &r, ProgSmem &sm, const HuffTable &t) {
  if (r.nbits < 16) wr_fill(r, sm);
  const uint32_t e = prog_lookup(t, (uint32_t)(r.buf >> 32));
  const uint32_t l = e >> 8;
  r.buf <<= l;
  r.nbits -= (int32_t)l;
  return e & 0xFFu;
}

// restart (libjpeg process_restart): drop the buffered bits, continue after the next RSTn
__device__ __forceinline__ void wr_restart(WReader &r, ProgSmem &sm) {
  r.buf = 0;
  r.nbits = 0;
  uint32_t q = r.p;
  while (q + 1 < r.len && !(wr_byte(r, sm, q) == 0xFF && (wr_byte(r, sm, q + 1) & 0xF8u) == 0xD0u)) q++;
  if (q + 1 < r.len) r.p = q + 2;
  r.marker = 0;
}

struct ProgState {
  int32_t pred[4];
  uint32_t eobrun;
};

// zigzag index k of a block (indices past 63 from corrupt runs land on 63,
// like libjpeg's jpeg_natural_order padding)
__device__ __forceinline__ uint32_t zz(uint32_t k) { return k < 63u ? k : 63u; }

// one block of the scan (libjpeg jdphuff.c decode_mcu_{DC,AC}_{first,refine})
__device__ __forceinline__ void prog_block(const ProgScan &sc, ProgSmem &sm, WReader &r, ProgState &ps, uint32_t ci,
                                           int16_t *blk, uint64_t nz, uint64_t *mask) {
  const uint32_t ss = sc.ss, se = sc.se, al = sc.al;
  if (ss == 0) {
    if (sc.ah == 0) {  // DC first
      const uint32_t s = wr_sym(r, sm, sm.tabs[ci]) & 15u;
      const int32_t diff = s ? huff_extend((int32_t)wr_get(r, sm, s), (int32_t)s) : 0;
      const int32_t p = (ci == 0 ? ps.pred[0] : ci == 1 ? ps.pred[1] : ci == 2 ? ps.pred[2] : ps.pred[3]) + diff;
      ps.pred[0] = ci == 0 ? p : ps.pred[0];
      ps.pred[1] = ci == 1 ? p : ps.pred[1];
      ps.pred[2] = ci == 2 ? p : ps.pred[2];
      ps.pred[3] = ci == 3 ? p : ps.pred[3];
      blk[0] = (int16_t)((uint32_t)p << al);
    } else if (wr_get(r, sm, 1)) {  // DC refine
      blk[0] = (int16_t)((int16_t)uni((uint32_t)(int32_t)blk[0]) | (int16_t)(1u << al));
    }
    return;
  }
  const HuffTable &ac = sm.tabs[0];
  if (sc.ah == 0) {  // AC first
    if (ps.eobrun > 0) {
      ps.eobrun--;
      return;
    }
    for (uint32_t k = ss; k <= se; k++) {
      const uint32_t rs = wr_sym(r, sm, ac);
      const uint32_t rr = rs >> 4, s = rs & 15u;
      if (s) {
        k += rr;
        const int32_t v = huff_extend((int32_t)wr_get(r, sm, s), (int32_t)s);
        blk[zz(k)] = (int16_t)((uint32_t)v << al);
      } else if (rr == 15) {
        k += 15;
      } else {
        ps.eobrun = (1u << rr) + wr_get(r, sm, rr) - 1u;
        break;
      }
    }
    return;
  }
  // AC refine.  Every position of the band that was nonzero before this
  // scan takes exactly one correction bit, in increasing position order
  // (libjpeg: the walk over "*thiscoef != 0" positions between symbols, and
  // the sweep to Se after an EOB), and coefficients this scan makes nonzero
  // always lie behind k.  So the decode consumes the correction bits of each
  // stretch of history-nonzero positions in one go (popcount of the block's
  // history mask) and records them as one bit string; the lanes map bit i to
  // the i-th history-nonzero position after the chunk.  A block inside an EOB
  // run costs O(1) instead of one step per coefficient.
  const uint64_t band = (se < 63 ? (2ull << se) - 1ull : ~0ull) & ~((1ull << ss) - 1ull);
  const uint64_t nzb = nz & band;
  uint64_t cbits = 0, nwp = 0, nwn = 0;
  uint32_t ccount = 0;
  auto take = [&](uint32_t c) {  // c <= 63 correction bits, appended in stream order
    if (c == 0) return;
    uint64_t v;
    if (c > 32) {
      const uint64_t hi = wr_get(r, sm, c - 32);
      v = (hi << 32) | wr_get(r, sm, 32);
    } else {
      v = wr_get(r, sm, c);
    }
    cbits = (cbits << c) | v;  // ccount + c <= 63: bits already taken are never shifted out
    ccount += c;
  };
  uint32_t k = ss;
  if (ps.eobrun == 0) {
    for (; k <= se; k++) {
      const uint32_t rs = wr_sym(r, sm, ac);
      uint32_t rr = rs >> 4;
      int32_t s = (int32_t)(rs & 15u);
      if (s) {
        s = wr_get(r, sm, 1) ? 1 : -1;
      } else if (rr != 15) {
        ps.eobrun = (1u << rr) + wr_get(r, sm, rr);
        break;
      }
      // skip rr history-zero positions from k; stop on the next one
      const uint64_t from = ~0ull << k;
      uint64_t z = ~nz & band & from;
      for (uint32_t i = 0; i < rr && z; i++) z &= z - 1ull;
      if (z) {
        const uint32_t pos = (uint32_t)__builtin_ctzll(z);
        take((uint32_t)__builtin_popcountll(nzb & from & ((1ull << pos) - 1ull)));
        k = pos;
      } else {  // ran past Se
        take((uint32_t)__builtin_popcountll(nzb & from));
        k = se + 1;
      }
      if (s > 0) nwp |= 1ull << zz(k);
      if (s < 0) nwn |= 1ull << zz(k);
    }
  }
  if (ps.eobrun > 0) {
    if (k <= se) take((uint32_t)__builtin_popcountll(nzb & (~0ull << k)));
    ps.eobrun--;
  }
  mask[0] = cbits;
  mask[1] = nwp;
  mask[2] = nwn;
  mask[3] = ccount;
}

// global block index of block j (in scan order) of unit (MCU) m; ci = scan component
__device__ __forceinline__ uint32_t prog_unit_block(const ImageDesc &im, const ProgScan &sc, uint32_t m, uint32_t j,
                                                    uint32_t &ci) {
  if (sc.ns == 1) {
    const uint32_t c = sc.comp[0];
    ci = 0;
    if (im.ncomp == 1) {
      const uint32_t nbx = (im.cdsw[0] + 7) / 8;
      return (m / nbx) * im.cbw[0] + m % nbx;
    }
    const uint32_t nbx = (im.cdsw[c] + 7) / 8;
    const uint32_t by = m / nbx, bx = m - by * nbx, h = im.ch[c], v = im.cv[c];
    return ((by / v) * im.mcux + bx / h) * im.bpm + im.cfirst[c] + (by % v) * h + bx % h;
  }
  uint32_t i = 0;
  for (; i + 1 < sc.ns; i++) {
    const uint32_t nb = im.ch[sc.comp[i]] * im.cv[sc.comp[i]];
    if (j < nb) break;
    j -= nb;
  }
  ci = i;
  const uint32_t c = sc.comp[i];
  return m * im.bpm + im.cfirst[c] + j;  // blocks of c within an MCU are in (v, h) raster order
}

__global__ __launch_bounds__(64) void k_prog_scan(const ImageDesc *__restrict__ imgs,
                                                  const ProgScan *__restrict__ scans,
                                                  const WgItem *__restrict__ list, const HuffTable *__restrict__ pool) {
  __shared__ ProgSmem sm;
  const ProgScan &sc = scans[list[blockIdx.x].item0];
  const ImageDesc &im = imgs[sc.image];
  const uint32_t lane = threadIdx.x;
  // tables: one per scan component (DC first) or the AC table
  {
    const uint32_t words = (uint32_t)(sizeof(HuffTable) / 4);
    const uint32_t nt = (sc.ss == 0) ? (sc.ah == 0 ? sc.ns : 0) : 1;
    for (uint32_t t = 0; t < nt; t++) {
      const uint32_t *src = (const uint32_t *)&pool[sc.ss == 0 ? sc.dc[t] : sc.ac];
      for (uint32_t w = lane; w < words; w += 64) ((uint32_t *)&sm.tabs[t])[w] = src[w];
    }
  }
  DG_GLOBAL int16_t *coef = gp<int16_t>(im.coef);
  // units: MCUs of the scan (a single block when ns == 1)
  uint32_t bpmu = 1, nunits;
  if (sc.ns == 1) {
    nunits = ((im.cdsw[sc.comp[0]] + 7) / 8) * ((im.cdsh[sc.comp[0]] + 7) / 8);
  } else {
    bpmu = 0;
    for (uint32_t i = 0; i < sc.ns; i++) bpmu += im.ch[sc.comp[i]] * im.cv[sc.comp[i]];
    nunits = im.mcux * im.mcuy;
  }
  const uint32_t upc = kPBlk / bpmu;  // units per chunk
  const bool refine = sc.ah != 0;
  WReader r;
  r.d = sc.data;
  r.len = sc.len;
  r.p = 0;
  r.buf = 0;
  r.nbits = 0;
  r.marker = 0;
  wr_refill(r, sm, 0);
  ProgState ps = {{0, 0, 0, 0}, 0};
  uint32_t since = 0;
  const uint32_t R = sc.restart;
  for (uint32_t u0 = 0; u0 < nunits; u0 += upc) {
    const uint32_t nu = nunits - u0 < upc ? nunits - u0 : upc;
    const uint32_t nb = nu * bpmu;
    // stage this chunk's blocks (lane = block slot)
    uint32_t g = 0, lci;
    if (lane < nb) {
      g = prog_unit_block(im, sc, u0 + lane / bpmu, lane % bpmu, lci);
      u32x4 *dst = (u32x4 *)sm.blk[lane];
      const DG_GLOBAL u32x4 *src = (const DG_GLOBAL u32x4 *)(coef + (size_t)g * 64);
#pragma unroll
      for (int q = 0; q < 8; q++) dst[q] = refine ? src[q] : u32x4{0u, 0u, 0u, 0u};
      if (refine) {
        uint64_t m = 0;
        for (uint32_t k = 0; k < 64; k++) m |= (uint64_t)(sm.blk[lane][k] != 0) << k;
        sm.nzm[lane] = m;
      }
    }
    __syncthreads();
    for (uint32_t u = 0; u < nu; u++) {
      if (R && since == R) {
        wr_restart(r, sm);
        ps = ProgState{{0, 0, 0, 0}, 0};
        since = 0;
      }
      for (uint32_t j = 0; j < bpmu; j++) {
        uint32_t ci = 0;
        if (sc.ns > 1) prog_unit_block(im, sc, 0, j, ci);
        const uint32_t slot = u * bpmu + j;
        uint64_t mk[4];
        prog_block(sc, sm, r, ps, ci, sm.blk[slot], refine ? uni64(sm.nzm[slot]) : 0ull, mk);
        if (refine && sc.ss > 0) {
          sm.cor[slot] = mk[0];
          sm.nwp[slot] = mk[1];
          sm.nwn[slot] = mk[2];
          sm.ncor[slot] = (uint32_t)mk[3];
        }
      }
      since++;
    }
    __syncthreads();
    // AC refine: apply the recorded corrections and new coefficients
    if (lane < nb && refine && sc.ss > 0) {
      const int32_t p1 = 1 << sc.al, m1 = -(1 << sc.al);
      int16_t *bk = sm.blk[lane];
      const uint64_t bits = sm.cor[lane];
      const uint32_t ss = sc.ss, se = sc.se;
      const uint64_t band = (se < 63 ? (2ull << se) - 1ull : ~0ull) & ~((1ull << ss) - 1ull);
      int32_t i = (int32_t)sm.ncor[lane] - 1;  // bit of the lowest history-nonzero position
      for (uint64_t m = sm.nzm[lane] & band; m && i >= 0; m &= m - 1ull, i--) {
        if (!((bits >> i) & 1u)) continue;
        const uint32_t pos = (uint32_t)__builtin_ctzll(m);
        const int32_t v = bk[pos];
        if ((v & p1) == 0) bk[pos] = (int16_t)(v >= 0 ? v + p1 : v + m1);
      }
      for (uint64_t m = sm.nwp[lane]; m; m &= m - 1ull) bk[__builtin_ctzll(m)] = (int16_t)p1;
      for (uint64_t m = sm.nwn[lane]; m; m &= m - 1ull) bk[__builtin_ctzll(m)] = (int16_t)m1;
    }
    // write back the scan's band of each block
    if (lane < nb) {
      DG_GLOBAL int16_t *dst = coef + (size_t)g * 64;
      for (uint32_t k = sc.ss; k <= sc.se; k++) dst[k] = sm.blk[lane][k];
    }
  }
}

// ------------------------------------------------------------ launchers

void launch_prog_zero(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_prog_zero, dim3(nwg), dim3(256), 0, st, imgs, list);
}

void launch_prog_scan(hipStream_t st, const ImageDesc *imgs, const ProgScan *scans, const WgItem *list, uint32_t n,
                      const HuffTable *pool) {
  if (n) hipLaunchKernelGGL(k_prog_scan, dim3(n), dim3(64), 0, st, imgs, scans, list, pool);
}

}  // namespace dg
