// dg_png.hip — CDNA4 (gfx950) kernels of the PNG half of the decode stage and
// the RGBA handling around the resize (fast_image_resize mul_div_alpha).
//
//   k_png_gather    IDAT payloads -> one contiguous zlib stream per image
//   k_png_inflate   zlib/DEFLATE -> filtered scanlines, one wave per image
//   k_png_unfilter  scanline filters -> samples, one wave per image
//   k_png_expand    palette / sub-byte gray / tRNS -> 8-bit L, LA, RGB, RGBA
//   k_alpha         premultiply / divide by alpha, in place
//
// What they restate: png 0.18.0 + fdeflate 0.3.7 as image 0.25.9 drives them
// (EXPAND), the reference's decode step for PNG (worker_files.rs:8-17,
// worker_wds.rs:45); RFC 1950/1951 for the stream, PNG spec 9.2-9.4 for the
// filters.  oracle/png_oracle.c is the CPU restatement the tests compare to.
//
// DEFLATE is a serial bit stream: the symbol boundaries of a block are only
// known by decoding it, and a match may copy bytes produced a moment before.
// k_png_inflate therefore decodes wave-uniformly (every lane holds the same
// bit reader and table lookups are LDS broadcasts, so the control flow is
// scalar) and spends the 64 lanes on what is parallel: table construction,
// the byte copies of matches and literal runs, input prefetch and the output
// stream, which goes through a 64 KiB LDS ring (the 32 KiB DEFLATE window plus
// one flush unit) to HBM in 32 KiB coalesced bursts.  Parallelism across the
// batch comes from one wave per image.
#include <hip/hip_runtime.h>

#include "dg_types.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace dg {

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------ gather

__global__ __launch_bounds__(256) void k_png_gather(const GatherJob *__restrict__ jobs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const GatherJob j = jobs[it.image];
  const uint32_t b0 = it.item0 * kGatherPiece;
  const uint32_t e = j.len - b0 < kGatherPiece ? j.len : b0 + kGatherPiece;
  const DG_GLOBAL uint8_t *s = gp<const uint8_t>(j.src);
  DG_GLOBAL uint8_t *d = gp<uint8_t>(j.dst);
  for (uint32_t i = b0 + threadIdx.x; i < e; i += 256) d[i] = s[i];
}

// ------------------------------------------------------------ inflate

constexpr uint32_t kRing = 65536, kRingMask = kRing - 1;
constexpr uint32_t kFlush = 32768;     // ring -> HBM burst
constexpr uint32_t kWin = 1024;        // input window (32-bit words) in LDS
constexpr uint32_t kLitBits = 10, kDistBits = 8, kClBits = 7;

__constant__ uint16_t c_lbase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                     33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                     1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Canonical Huffman table in LDS.  lut[prefix] = (symbol << 4) | length for
// codes no longer than B bits, 0 for prefixes of longer codes (decoded by the
// bit-serial canonical walk over cnt/first/off/sym).
struct HTab {
  uint16_t *lut;
  uint16_t *sym;
  uint32_t *cnt;    // [16] codes per length
  uint32_t *first;  // [16] first canonical code of each length
  uint32_t *off;    // [16] index in sym of each length's first symbol
  uint32_t B;
};

struct InflateSmem {
  uint8_t ring[kRing];
  uint32_t win[kWin];
  uint16_t lut_l[1 << kLitBits], lut_d[1 << kDistBits], lut_c[1 << kClBits];
  uint16_t sym_l[288], sym_d[32], sym_c[20];
  uint32_t cnt[3][16], first[3][16], off[3][16], run[16];
  uint8_t lens[320];
  uint32_t flag;
};

// Builds `t` from lens[0..n) with all 64 lanes.  Returns false (uniform) for an
// over-subscribed code.
__device__ bool build_table(InflateSmem &sm, const uint8_t *lens, uint32_t n, HTab t) {
  const uint32_t lane = threadIdx.x;
  if (lane < 16) t.cnt[lane] = 0;
  __syncthreads();
  for (uint32_t s = lane; s < n; s += 64) {
    const uint32_t l = lens[s];
    if (l) atomicAdd(&t.cnt[l], 1u);
  }
  __syncthreads();
  if (lane == 0) {
    int left = 1;
    uint32_t code = 0, o = 0;
    bool ok = true;
    for (uint32_t l = 1; l < 16; l++) {
      left = 2 * left - (int)t.cnt[l];
      if (left < 0) ok = false;
      code = (code + t.cnt[l - 1]) << 1;
      if (l == 1) code = 0;
      t.first[l] = code;
      t.off[l] = o;
      sm.run[l] = o;
      o += t.cnt[l];
    }
    t.first[0] = 0;
    t.off[0] = 0;
    sm.flag = ok ? 1u : 0u;
  }
  __syncthreads();
  if (!uni(sm.flag)) return false;
  // sorted symbols: rank among equal lengths by ballot, chunk by chunk
  const uint64_t lt = (1ull << lane) - 1ull;
  for (uint32_t base = 0; base < n; base += 64) {
    const uint32_t s = base + lane;
    const uint32_t l = s < n ? lens[s] : 0u;
    for (uint32_t L = 1; L < 16; L++) {
      const uint64_t m = __ballot(l == L);
      if (m == 0) continue;
      const uint32_t r = sm.run[L];
      if (l == L) t.sym[r + (uint32_t)__popcll(m & lt)] = (uint16_t)s;
      __syncthreads();
      if (lane == 0) sm.run[L] = r + (uint32_t)__popcll(m);
      __syncthreads();
    }
  }
  __syncthreads();
  // first-level lookup, one entry per lane at a time
  for (uint32_t e = lane; e < (1u << t.B); e += 64) {
    uint16_t v = 0;
    const uint32_t rv = __builtin_bitreverse32(e);
    for (uint32_t L = 1; L <= t.B; L++) {
      const uint32_t c = rv >> (32 - L);
      const uint32_t k = c - t.first[L];
      if (k < t.cnt[L]) {
        v = (uint16_t)((t.sym[t.off[L] + k] << 4) | L);
        break;
      }
    }
    t.lut[e] = v;
  }
  __syncthreads();
  return true;
}

// Wave-uniform LSB-first bit reader over the LDS input window.
struct BitReader {
  uint64_t bb;      // bit buffer
  uint32_t nb;      // valid bits in bb
  uint32_t wnext;   // next word to load into bb
  uint32_t wbase;   // first word held by the window
  uint32_t zwords;  // words in the stream (the last one may be partial)
};

__device__ __forceinline__ void win_load(InflateSmem &sm, const DG_GLOBAL uint32_t *z, uint32_t zwords,
                                         uint32_t w0, uint32_t count) {
  for (uint32_t i = threadIdx.x; i < count; i += 64) {
    const uint32_t w = w0 + i;
    sm.win[w & (kWin - 1)] = w < zwords ? z[w] : 0u;
  }
  __syncthreads();
}

// Make sure bb holds at least 32 bits (all lanes, uniform control flow).
__device__ __forceinline__ void refill(InflateSmem &sm, BitReader &br, const DG_GLOBAL uint32_t *z) {
  if (br.nb >= 32) return;
  if (br.wnext + 2 > br.wbase + kWin) {  // slide the window by half
    win_load(sm, z, br.zwords, br.wbase + kWin, kWin / 2);
    br.wbase += kWin / 2;
  }
  const uint32_t w = uni(sm.win[br.wnext & (kWin - 1)]);
  br.bb |= (uint64_t)w << br.nb;
  br.nb += 32;
  br.wnext++;
}

__device__ __forceinline__ uint32_t getbits(BitReader &br, uint32_t k) {
  const uint32_t v = (uint32_t)br.bb & ((1u << k) - 1u);
  br.bb >>= k;
  br.nb -= k;
  return v;
}

// Decode one symbol (bb holds >= 15 bits).  Returns the symbol or 0xFFFF.
__device__ __forceinline__ uint32_t decode_sym(BitReader &br, const HTab &t) {
  const uint32_t peek = (uint32_t)br.bb;
  const uint32_t e = uni(t.lut[peek & ((1u << t.B) - 1u)]);
  if (e & 15u) {
    const uint32_t l = e & 15u;
    br.bb >>= l;
    br.nb -= l;
    return e >> 4;
  }
  const uint32_t rv = __builtin_bitreverse32(peek);
  for (uint32_t L = t.B + 1; L < 16; L++) {
    const uint32_t c = rv >> (32 - L);
    const uint32_t k = c - uni(t.first[L]);
    if (k < uni(t.cnt[L])) {
      br.bb >>= L;
      br.nb -= L;
      return uni(t.sym[uni(t.off[L]) + k]);
    }
  }
  return 0xFFFFu;
}

// ring[fp .. fp+n) -> out[fp .. fp+n), clamped to `want`
__device__ __forceinline__ void flush_ring(InflateSmem &sm, DG_GLOBAL uint8_t *out, uint32_t fp, uint32_t n,
                                           uint32_t want) {
  if (fp + n > want) n = want > fp ? want - fp : 0u;
  const uint32_t lane = threadIdx.x;
  if ((fp & 15u) == 0 && n == kFlush) {
    for (uint32_t i = lane * 16; i < n; i += 64 * 16) {
      const uint32_t r = (fp + i) & kRingMask;
      *(DG_GLOBAL u32x4 *)(out + fp + i) = *(const u32x4 *)(sm.ring + r);
    }
  } else {
    for (uint32_t i = lane; i < n; i += 64) out[fp + i] = sm.ring[(fp + i) & kRingMask];
  }
}

__global__ __launch_bounds__(64) void k_png_inflate(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  InflateSmem &sm = *reinterpret_cast<InflateSmem *>(smem_raw);
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  const PngDesc &pd = im.png;
  const uint32_t lane = threadIdx.x;
  const DG_GLOBAL uint32_t *z = gp<const uint32_t>(pd.zs);
  DG_GLOBAL uint8_t *out = gp<uint8_t>(pd.raw);
  const uint32_t want = uni(im.height * (pd.rowbytes + 1u));
  const uint32_t zlen = uni(pd.zlen);
  BitReader br;
  br.bb = 0;
  br.nb = 0;
  br.wnext = 0;
  br.wbase = 0;
  br.zwords = (zlen + 3u) / 4u;
  win_load(sm, z, br.zwords, 0, kWin);
  HTab tl{sm.lut_l, sm.sym_l, sm.cnt[0], sm.first[0], sm.off[0], kLitBits};
  HTab td{sm.lut_d, sm.sym_d, sm.cnt[1], sm.first[1], sm.off[1], kDistBits};
  HTab tc{sm.lut_c, sm.sym_c, sm.cnt[2], sm.first[2], sm.off[2], kClBits};
  uint32_t op = 0, fp = 0;  // output produced / flushed to HBM
  uint32_t nlit = 0;        // literals stashed in lanes [0, nlit) (positions op - nlit + lane)
  uint32_t litv = 0;
  int status = 0;
  const uint64_t limit_bits = (uint64_t)zlen * 8u;
  auto consumed = [&]() -> uint64_t { return (uint64_t)br.wnext * 32u - br.nb; };
  auto stash_flush = [&]() {
    if (nlit) {
      if (lane < nlit) sm.ring[(op - nlit + lane) & kRingMask] = (uint8_t)litv;
      nlit = 0;
    }
  };
  auto maybe_flush = [&]() {
    if (op - fp >= kFlush) {
      stash_flush();
      __syncthreads();
      flush_ring(sm, out, fp, kFlush, want);
      fp += kFlush;
    }
  };
  refill(sm, br, z);
  {
    const uint32_t cmf = getbits(br, 8), flg = getbits(br, 8);
    if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u)) status = 2;
  }
  bool last = false;
  while (!status && !last && op < want) {
    refill(sm, br, z);
    last = getbits(br, 1) != 0;
    const uint32_t type = getbits(br, 2);
    if (type == 3) {
      status = 2;
      break;
    }
    if (type == 0) {  // stored block: byte-align, LEN/NLEN, raw copy from the stream
      getbits(br, br.nb & 7u);
      refill(sm, br, z);
      const uint32_t len = getbits(br, 16), nlen = getbits(br, 16);
      if ((len ^ 0xFFFFu) != nlen) {
        status = 2;
        break;
      }
      const uint32_t pos = br.wnext * 4u - br.nb / 8u;  // next unread byte
      if ((uint64_t)pos + len > zlen) {
        status = 2;
        break;
      }
      stash_flush();
      const DG_GLOBAL uint8_t *zb = (const DG_GLOBAL uint8_t *)z;
      uint32_t done = 0;
      while (done < len && op < want) {
        uint32_t n = len - done;
        const uint32_t room = fp + kFlush + kFlush / 2 - op;  // keep op - fp below the ring's reach
        if (n > room) n = room;
        for (uint32_t j = lane; j < n; j += 64) sm.ring[(op + j) & kRingMask] = zb[pos + done + j];
        op += n;
        done += n;
        __syncthreads();
        while (op - fp >= kFlush) {
          flush_ring(sm, out, fp, kFlush, want);
          fp += kFlush;
          __syncthreads();
        }
      }
      // reposition the reader after the block
      const uint32_t np = pos + len;
      br.bb = 0;
      br.nb = 0;
      br.wnext = np / 4u;
      if (br.wnext < br.wbase || br.wnext + 2 > br.wbase + kWin) {
        br.wbase = br.wnext;
        win_load(sm, z, br.zwords, br.wbase, kWin);
      }
      refill(sm, br, z);
      getbits(br, (np & 3u) * 8u);
      continue;
    }
    // code lengths
    if (type == 1) {
      for (uint32_t s = lane; s < 320; s += 64)
        sm.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;  // 288.. = distances
      __syncthreads();
      build_table(sm, sm.lens, 288, tl);
      build_table(sm, sm.lens + 288, 30, td);
    } else {
      refill(sm, br, z);
      const uint32_t nlen = getbits(br, 5) + 257, ndist = getbits(br, 5) + 1, ncode = getbits(br, 4) + 4;
      if (nlen > 286 || ndist > 30) {
        status = 2;
        break;
      }
      if (lane < 19) sm.lens[lane] = 0;
      __syncthreads();
      for (uint32_t i = 0; i < ncode; i++) {
        refill(sm, br, z);
        const uint32_t v = getbits(br, 3);
        if (lane == 0) sm.lens[c_clorder[i]] = (uint8_t)v;
      }
      __syncthreads();
      if (!build_table(sm, sm.lens, 19, tc)) {
        status = 2;
        break;
      }
      uint32_t i = 0, prev = 0;
      const uint32_t total = nlen + ndist;
      while (i < total) {
        refill(sm, br, z);
        const uint32_t s = decode_sym(br, tc);
        if (s < 16) {
          if (lane == 0) sm.lens[i] = (uint8_t)s;
          prev = s;
          i++;
          continue;
        }
        uint32_t rep, v = 0;
        if (s == 16) {
          if (i == 0) {
            status = 2;
            break;
          }
          v = prev;
          rep = 3 + getbits(br, 2);
        } else if (s == 17) {
          rep = 3 + getbits(br, 3);
        } else if (s == 18) {
          rep = 11 + getbits(br, 7);
        } else {
          status = 2;
          break;
        }
        if (i + rep > total) {
          status = 2;
          break;
        }
        if (lane < rep) sm.lens[i + lane] = (uint8_t)v;
        if (lane + 64 < rep) sm.lens[i + 64 + lane] = (uint8_t)v;
        if (lane + 128 < rep) sm.lens[i + 128 + lane] = (uint8_t)v;
        prev = v;
        i += rep;
      }
      if (status) break;
      __syncthreads();
      if (uni(sm.lens[256]) == 0) {
        status = 2;
        break;
      }
      // distance lengths must sit at 288.. for the shared layout: move them
      uint8_t dl = 0;
      if (lane < ndist) dl = sm.lens[nlen + lane];
      __syncthreads();
      for (uint32_t s = nlen + lane; s < 288; s += 64) sm.lens[s] = 0;
      __syncthreads();
      if (lane < 32) sm.lens[288 + lane] = lane < ndist ? dl : 0;
      __syncthreads();
      if (!build_table(sm, sm.lens, nlen, tl) || !build_table(sm, sm.lens + 288, ndist, td)) {
        status = 2;
        break;
      }
    }
    // symbols
    for (;;) {
      refill(sm, br, z);
      const uint32_t s = decode_sym(br, tl);
      if (s < 256) {
        if (lane == nlit) litv = s;
        nlit++;
        op++;
        if (nlit == 64) stash_flush();
        if (op >= want) break;
        maybe_flush();
        continue;
      }
      if (s == 256) break;
      if (s > 285) {
        status = 2;
        break;
      }
      const uint32_t len = c_lbase[s - 257] + getbits(br, c_lext[s - 257]);
      refill(sm, br, z);
      const uint32_t ds = decode_sym(br, td);
      if (ds >= 30) {
        status = 2;
        break;
      }
      refill(sm, br, z);
      const uint32_t dist = c_dbase[ds] + getbits(br, c_dext[ds]);
      if (dist > op) {
        status = 2;
        break;
      }
      stash_flush();
      // every source byte lies before `op`: one read + one write per lane and 64 bytes
      const uint32_t q = op, src0 = op - dist;
      const float rcp = 1.0f / (float)dist;
      for (uint32_t j = lane; j < len; j += 64) {
        uint32_t k = j;
        if (dist < len) {
          uint32_t qt = (uint32_t)((float)j * rcp);
          k = j - qt * dist;
          if (k >= dist) k -= dist;
        }
        const uint8_t v = sm.ring[(src0 + k) & kRingMask];
        sm.ring[(q + j) & kRingMask] = v;
      }
      op += len;
      if (op >= want) break;
      if (consumed() > limit_bits + 64) {
        status = 2;
        break;
      }
      maybe_flush();
    }
    if (consumed() > limit_bits + 64) status = 2;
  }
  if (!status && op < want) status = 2;  // stream ended before the last scanline
  stash_flush();
  __syncthreads();
  // final flush: [fp, min(op, want))
  while (fp < op && fp < want) {
    const uint32_t n = op - fp < kFlush ? op - fp : kFlush;
    flush_ring(sm, out, fp, n, want);
    fp += n;
  }
  if (status && lane == 0) im.status = status;
}

// ------------------------------------------------------------ unfilter

// One wave per image.  Rows are taken 64 at a time, lane l owning row y0 + l,
// on a diagonal: at step t lane l unfilters pixel x = t - l, so the pixel
// above (row y-1, x) and above-left (x-1) were produced by lane l-1 at steps
// t-1 and t-2 and arrive by a lane shuffle; the left pixel is the lane's own
// previous result.  Lane 0 reads the band's previous row from memory.
// Samples of up to 4 bytes per filter unit (8-bit L/LA/RGB/RGBA; 1 for
// palette and sub-byte gray) travel packed in one dword.
__device__ __forceinline__ uint32_t paeth_b(uint32_t a, uint32_t b, uint32_t c) {
  const int p = (int)a + (int)b - (int)c;
  const int pa = abs(p - (int)a), pb = abs(p - (int)b), pc = abs(p - (int)c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

__device__ __forceinline__ uint32_t shfl_up1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((threadIdx.x + 63u) & 63u) << 2), (int)v);
}

__global__ __launch_bounds__(64) void k_png_unfilter(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  const PngDesc &pd = im.png;
  if (im.status) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t rb = pd.rowbytes, bpp = pd.bpp, us = pd.ustride, H = im.height;
  const uint32_t units = (rb + bpp - 1) / bpp;  // rowbytes is a multiple of bpp for 8-bit samples
  const DG_GLOBAL uint8_t *raw = gp<const uint8_t>(pd.raw);
  DG_GLOBAL uint8_t *unf = gp<uint8_t>(pd.unf);
  int bad = 0;
  for (uint32_t y0 = 0; y0 < H; y0 += 64) {
    const uint32_t y = y0 + lane;
    const bool active = y < H;
    const DG_GLOBAL uint8_t *r = raw + (size_t)y * (rb + 1);
    DG_GLOBAL uint8_t *o = unf + (size_t)y * us;
    const DG_GLOBAL uint8_t *prow = y > 0 ? unf + (size_t)(y - 1) * us : nullptr;
    uint32_t f = active ? r[0] : 0u;
    if (f > 4) {
      bad = 1;
      f = 0;
    }
    r++;
    uint32_t cur = 0, prev = 0, prev2 = 0;  // results of steps t, t-1, t-2 (packed bytes)
    const uint32_t nsteps = units + 63;
    for (uint32_t t = 0; t < nsteps; t++) {
      // neighbour row: lane l-1's results of steps t-1 (above) and t-2 (above-left)
      uint32_t up = shfl_up1(prev), ul = shfl_up1(prev2);
      const int32_t x = (int32_t)t - (int32_t)lane;
      if (active && x >= 0 && (uint32_t)x < units) {
        const uint32_t b0 = (uint32_t)x * bpp;
        if (lane == 0) {  // previous band's last row comes from memory
          up = 0;
          ul = 0;
          if (prow) {
            for (uint32_t k = 0; k < bpp; k++) up |= (uint32_t)prow[b0 + k] << (8 * k);
            if (x > 0)
              for (uint32_t k = 0; k < bpp; k++) ul |= (uint32_t)prow[b0 - bpp + k] << (8 * k);
          }
        } else if (y == 0) {
          up = ul = 0;
        }
        if (x == 0) ul = 0;
        const uint32_t left = x > 0 ? prev : 0u;
        uint32_t v = 0;
        for (uint32_t k = 0; k < bpp; k++) {
          const uint32_t sh = 8 * k;
          const uint32_t a = (left >> sh) & 0xFFu, b = (up >> sh) & 0xFFu, c = (ul >> sh) & 0xFFu;
          uint32_t pr;
          switch (f) {
            case 0: pr = 0; break;
            case 1: pr = a; break;
            case 2: pr = b; break;
            case 3: pr = (a + b) >> 1; break;
            default: pr = paeth_b(a, b, c); break;
          }
          const uint32_t bx = b0 + k;
          const uint32_t rv = bx < rb ? (uint32_t)r[bx] : 0u;
          v |= ((rv + pr) & 0xFFu) << sh;
        }
        for (uint32_t k = 0; k < bpp; k++)
          if (b0 + k < rb) o[b0 + k] = (uint8_t)(v >> (8 * k));
        cur = v;
      } else {
        cur = 0;
      }
      prev2 = prev;
      prev = cur;
    }
    // the next band's lane 0 reads this band's last row from memory
    __threadfence();
    __syncthreads();
  }
  if (__ballot(bad) && lane == 0) im.status = 2;
}

// ------------------------------------------------------------ expand

// One pixel per thread: palette -> RGB(A), 1/2/4-bit gray -> 8-bit (x 255/(2^d-1)),
// tRNS key -> alpha (png Transformations::EXPAND).
__global__ __launch_bounds__(256) void k_png_expand(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const PngDesc &pd = im.png;
  const uint32_t idx = it.item0 + threadIdx.x;
  const uint32_t W = im.width;
  if (idx >= W * im.height) return;
  const uint32_t y = idx / W, x = idx - y * W;
  const DG_GLOBAL uint8_t *r = gp<const uint8_t>(pd.unf) + (size_t)y * pd.ustride;
  const uint32_t C = im.dec_c;
  DG_GLOBAL uint8_t *o = gp<uint8_t>(im.pix) + (size_t)y * im.pix_stride + (size_t)x * C;
  const uint32_t dp = pd.depth;
  if (pd.ctype == 0 || pd.ctype == 3) {
    uint32_t v;
    if (dp == 8) {
      v = r[x];
    } else {
      const uint32_t bit = x * dp;
      v = ((uint32_t)r[bit >> 3] >> (8 - dp - (bit & 7))) & ((1u << dp) - 1u);
    }
    if (pd.ctype == 3) {
      const DG_GLOBAL uint8_t *pe = gp<const uint8_t>(pd.pal) + 4 * v;
      o[0] = pe[0];
      o[1] = pe[1];
      o[2] = pe[2];
      if (C == 4) o[3] = pe[3];
    } else {
      o[0] = (uint8_t)(v * (255u / ((1u << dp) - 1u)));
      if (C == 2) o[1] = v == pd.trns[0] ? 0 : 255;
    }
  } else {  // RGB with a tRNS key
    const DG_GLOBAL uint8_t *p = r + 3 * (size_t)x;
    const uint32_t a = p[0], b = p[1], c = p[2];
    o[0] = (uint8_t)a;
    o[1] = (uint8_t)b;
    o[2] = (uint8_t)c;
    o[3] = (a == pd.trns[0] && b == pd.trns[1] && c == pd.trns[2]) ? 0 : 255;
  }
}

// ------------------------------------------------------------ alpha

// fast_image_resize 5.5.0 alpha handling restated (SURVEY Appendix B2,
// unpinned: the crate is not present offline): multiply = mul_div_255
// (rounded a*b/255), divide = v * recip(a) with recip = round(255*2^8/a),
// rounded and clamped; alpha 0 divides to 0.
__device__ __forceinline__ uint32_t mul_div_255(uint32_t a, uint32_t b) {
  const uint32_t t = a * b + 128u;
  return (t + (t >> 8)) >> 8;
}
__device__ __forceinline__ uint32_t div_alpha(uint32_t v, uint32_t a) {
  if (a == 0) return 0;
  const uint32_t recip = ((255u << 9) / a + 1u) >> 1;
  const uint32_t r = (v * recip + 128u) >> 8;
  return r > 255u ? 255u : r;
}

__global__ __launch_bounds__(256) void k_alpha(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                               int point) {
  const WgItem it = list[blockIdx.x];
  const ImageDesc &im = imgs[it.image];
  if (im.status) return;
  const AlphaOp &ao = im.aop[point & 0xFF];
  if ((point >> 8) && ao.on_decoded) return;  // resync round: the decoded image is already done
  const uint32_t idx = it.item0 + threadIdx.x;
  if (idx >= ao.width * ao.rows) return;
  const uint32_t C = im.dec_c;
  const uint32_t y = idx / ao.width, x = idx - y * ao.width;
  DG_GLOBAL uint8_t *p = gp<uint8_t>(ao.buf) + (size_t)y * ao.stride + (size_t)x * C;
  uint32_t v[3] = {0, 0, 0};
  const uint32_t nc = C - 1;  // colour channels: 1 (LA) or 3 (RGBA)
#pragma unroll
  for (uint32_t c = 0; c < 3; c++)
    if (c < nc) v[c] = p[c];
  const uint32_t a = p[nc];
  for (uint32_t prog = ao.prog; prog; prog >>= 2) {
    const uint32_t op = prog & 3u;
#pragma unroll
    for (uint32_t c = 0; c < 3; c++) v[c] = op == 1 ? mul_div_255(v[c], a) : div_alpha(v[c], a);
  }
#pragma unroll
  for (uint32_t c = 0; c < 3; c++)
    if (c < nc) p[c] = (uint8_t)v[c];
}

// ------------------------------------------------------------ launchers

void launch_png_gather(hipStream_t st, const GatherJob *jobs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_png_gather, dim3(nwg), dim3(256), 0, st, jobs, list);
}
void launch_png_inflate(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  static bool attr = false;  // > 64 KiB of dynamic LDS
  if (!attr) {
    hipFuncSetAttribute((const void *)k_png_inflate, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)sizeof(InflateSmem));
    attr = true;
  }
  if (nwg)
    hipLaunchKernelGGL(k_png_inflate, dim3(nwg), dim3(64), sizeof(InflateSmem), st, imgs, list);
}
void launch_png_unfilter(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_png_unfilter, dim3(nwg), dim3(64), 0, st, imgs, list);
}
void launch_png_expand(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_png_expand, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_alpha(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int point) {
  if (nwg) hipLaunchKernelGGL(k_alpha, dim3(nwg), dim3(256), 0, st, imgs, list, point);
}
size_t png_inflate_smem() { return sizeof(InflateSmem); }

}  // namespace dg
