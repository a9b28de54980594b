// dg_png.hip — CDNA4 (gfx950) kernels of the PNG half of the decode stage and
// the RGBA handling around the resize (fast_image_resize mul_div_alpha).
//
//   k_png_gather    IDAT payloads -> one contiguous zlib stream per image
//   k_png_inflate   zlib/DEFLATE -> filtered scanlines, one wave per image
//   k_png_unfilter  scanline filters -> samples, one wave per 64-row band
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
#include <type_traits>
#include <hip/hip_runtime.h>

#include "dg_types.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace dg {

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------ gather

// An IDAT chunk's bytes into the image's contiguous zlib stream.  Both ends
// sit at arbitrary byte offsets (chunk headers in the file, cumulative IDAT
// lengths in the stream), so a thread stores 16-byte-aligned destination
// chunks built from five aligned source dwords (v_alignbyte); only the
// misaligned head and the tail go byte by byte.  (Byte loads and stores for
// every byte kept ~190 K waves resident per configs[4] batch.)  The source
// dword reads end at most 4 bytes past the chunk: inside the PNG file, whose
// IEND chunk follows the last IDAT.
__global__ __launch_bounds__(256) void k_png_gather(const GatherJob *__restrict__ jobs, const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  const GatherJob j = jobs[it.image];
  const uint32_t b0 = it.item0 * kGatherPiece;
  const uint32_t e = j.len - b0 < kGatherPiece ? j.len : b0 + kGatherPiece;
  const DG_GLOBAL uint8_t *s = gp<const uint8_t>(j.src);
  DG_GLOBAL uint8_t *d = gp<uint8_t>(j.dst);
  const uint32_t t = threadIdx.x;
  const uint32_t lead = (16u - (uint32_t)((j.dst + b0) & 15u)) & 15u;
  const uint32_t a0 = b0 + lead < e ? b0 + lead : e;  // first 16-byte-aligned destination offset
  const uint32_t nb = (e - a0) >> 4;                 // whole 16-byte chunks
  if (t < a0 - b0) d[b0 + t] = s[b0 + t];
  const uint32_t a1 = a0 + nb * 16u;
  if (t < e - a1) d[a1 + t] = s[a1 + t];
  for (uint32_t k = t; k < nb; k += 256) {
    const uint32_t o = a0 + 16u * k;
    const uint64_t sa = j.src + o;
    const uint32_t r = (uint32_t)sa & 3u;
    const DG_GLOBAL uint32_t *w = gp<const uint32_t>(sa - r);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(w1, w0, r);
    v.y = __builtin_amdgcn_alignbyte(w2, w1, r);
    v.z = __builtin_amdgcn_alignbyte(w3, w2, r);
    v.w = __builtin_amdgcn_alignbyte(w4, w3, r);
    *(DG_GLOBAL u32x4 *)(d + o) = v;
  }
}

// ------------------------------------------------------------ inflate

// The serial inflate writes every output byte through to HBM as it makes it
// (a wave's 64 consecutive bytes: one coalesced store) and keeps only the
// 32 KiB deflate window in LDS (round 5: a 64 KiB ring flushed in 32 KiB
// bursts held 74 KiB of LDS per workgroup, and the masks' workgroups waited
// to be dispatched behind the chunk decode and the unfilter).
constexpr uint32_t kRing = 32768, kRingMask = kRing - 1;
constexpr uint32_t kWin = 1024;        // input window (32-bit words) in LDS
constexpr uint32_t kLitBits = 10, kDistBits = 8, kClBits = 7;

// base | extra bits << 16 of each length / distance symbol: one dword, so a
// wave-uniform index reads it with a scalar load
__constant__ uint32_t c_lenx[29] = {
    3,  4,  5,  6,  7,  8,  9,  10, 11 | 1u << 16,  13 | 1u << 16,  15 | 1u << 16,  17 | 1u << 16,  19 | 2u << 16,
    23 | 2u << 16,  27 | 2u << 16,  31 | 2u << 16,  35 | 3u << 16,  43 | 3u << 16,  51 | 3u << 16,  59 | 3u << 16,
    67 | 4u << 16,  83 | 4u << 16,  99 | 4u << 16,  115 | 4u << 16, 131 | 5u << 16, 163 | 5u << 16, 195 | 5u << 16,
    227 | 5u << 16, 258};
__constant__ uint32_t c_distx[30] = {
    1,  2,  3,  4,  5 | 1u << 16,  7 | 1u << 16,  9 | 2u << 16,  13 | 2u << 16,  17 | 3u << 16,  25 | 3u << 16,
    33 | 4u << 16,  49 | 4u << 16,  65 | 5u << 16,  97 | 5u << 16,  129 | 6u << 16,  193 | 6u << 16,
    257 | 7u << 16,  385 | 7u << 16,  513 | 8u << 16,  769 | 8u << 16,  1025 | 9u << 16,  1537 | 9u << 16,
    2049 | 10u << 16,  3073 | 10u << 16,  4097 | 11u << 16,  6145 | 11u << 16,  8193 | 12u << 16,
    12289 | 12u << 16,  16385 | 13u << 16,  24577 | 13u << 16};
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

// The reader state is wave-uniform by construction; re-asserting it keeps the
// compiler from carrying it in VGPRs after the lane-dependent stores (it then
// branches on SCC and reads the symbol tables with scalar loads).
__device__ __forceinline__ void br_uni(BitReader &br) {
  br.bb = ((uint64_t)uni((uint32_t)(br.bb >> 32)) << 32) | uni((uint32_t)br.bb);
  br.nb = uni(br.nb);
  br.wnext = uni(br.wnext);
  br.wbase = uni(br.wbase);
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

// mode 0: streams too small to chunk (launched beside the chunked kernels);
// 1: images the chunked path gave up on (pd.serial, after k_inf_resolve);
// 2: both (one launch after the chunked kernels)
__device__ __forceinline__ void inflate_image(InflateSmem &sm, ImageDesc &im);

// mode 1 runs on up to one workgroup per CU that claim list entries from a
// work counter (BatchFlags::png_next) until the list is exhausted: the
// images the chunked path gave up on are rare (none in the configs[4] pool),
// and a workgroup per image -- each asking for ~41 KiB of LDS while the
// chunk decode and the unfilter hold most of it -- kept 3-10 ms of mostly
// empty workgroups waiting to be dispatched on every batch's critical path.
// A batch whose streams the chunked path cannot start in (stored or
// fixed-Huffman blocks only) still gets one workgroup per fallback image, up
// to one per CU (a fixed 4 workgroups serialised such batches).
// The wave raises its issue priority: one wave's serial chain per image, on
// the batch's critical path, sharing its SIMD with the throughput kernels of
// the other batches in flight (a 33 ms mask took 83 ms among them).
__global__ __launch_bounds__(64) void k_png_inflate(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                                    uint32_t n, int mode, BatchFlags *flags) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  InflateSmem &sm = *reinterpret_cast<InflateSmem *>(smem_raw);
  __shared__ uint32_t claim;
  __builtin_amdgcn_s_setprio(3);
  if (mode != 1) {  // modes 0 / 2: one image per workgroup
    ImageDesc &im = imgs[list[blockIdx.x].image];
    const PngDesc &pd = im.png;
    const bool take = mode == 0 ? pd.nchunks == 0 : !(pd.nchunks && !pd.serial);
    if (take) inflate_image(sm, im);
    return;
  }
  for (;;) {  // every workgroup exits once the counter passes n
    if (threadIdx.x == 0) claim = atomicAdd(&flags->png_next, 1u);
    __syncthreads();
    const uint32_t i = claim;
    __syncthreads();
    if (i >= n) return;
    ImageDesc &im = imgs[list[i].image];
    const PngDesc &pd = im.png;
    if (!(pd.nchunks && pd.serial)) continue;
    inflate_image(sm, im);
    __syncthreads();
  }
}

__device__ __forceinline__ void inflate_image(InflateSmem &sm, ImageDesc &im) {
  const PngDesc &pd = im.png;
  const uint32_t lane = threadIdx.x;
  const DG_GLOBAL uint32_t *z = gp<const uint32_t>(pd.zs);
  DG_GLOBAL uint8_t *out = gp<uint8_t>(pd.raw);
  const uint32_t want = uni(pd.rawlen);
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
  uint32_t op = 0;  // output produced (in HBM and the window)
  uint32_t nlit = 0;        // literals stashed in lanes [0, nlit) (positions op - nlit + lane)
  uint32_t litv = 0;
  int status = 0;
  const uint64_t limit_bits = (uint64_t)zlen * 8u;
  auto consumed = [&]() -> uint64_t { return (uint64_t)br.wnext * 32u - br.nb; };
  auto stash_flush = [&]() {
    if (nlit) {
      if (lane < nlit) {
        const uint32_t o = op - nlit + lane;
        sm.ring[o & kRingMask] = (uint8_t)litv;
        if (o < want) out[o] = (uint8_t)litv;
      }
      nlit = 0;
    }
  };
  refill(sm, br, z);
  {
    const uint32_t cmf = getbits(br, 8), flg = getbits(br, 8);
    if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u)) status = 2;
  }
  bool last = false;
  while (!status && !last && op < want) {
    br_uni(br);
    op = uni(op);
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
      // (a later byte of a block longer than the window lands in its slot
      // after the earlier one: same lane, later iteration)
      for (uint32_t j = lane; j < len; j += 64) {
        const uint8_t v = zb[pos + j];
        sm.ring[(op + j) & kRingMask] = v;
        if (op + j < want) out[op + j] = v;
      }
      op += len;
      __syncthreads();
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
      br_uni(br);
      op = uni(op);
      nlit = uni(nlit);
      refill(sm, br, z);
      const uint32_t s = decode_sym(br, tl);
      if (s < 256) {
        if (lane == nlit) litv = s;
        nlit++;
        op++;
        if (nlit == 64) stash_flush();
        if (op >= want) break;
        continue;
      }
      if (s == 256) break;
      if (s > 285) {
        status = 2;
        break;
      }
      const uint32_t lx = c_lenx[s - 257];
      const uint32_t len = (lx & 0xFFFFu) + getbits(br, lx >> 16);
      refill(sm, br, z);
      const uint32_t ds = decode_sym(br, td);
      if (ds >= 30) {
        status = 2;
        break;
      }
      refill(sm, br, z);
      const uint32_t dx = c_distx[ds];
      const uint32_t dist = (dx & 0xFFFFu) + getbits(br, dx >> 16);
      if (dist > op) {
        status = 2;
        break;
      }
      stash_flush();
      // every source byte lies before `op` (an overlapping copy repeats the
      // first `dist` bytes), so no read sees a byte this match writes.
      // Branches are wave-uniform.
      const uint32_t q = op, src0 = op - dist, rounds = (len + 63u) >> 6;
      if (dist == 1u) {  // run of one byte (masks, flat rows): one broadcast read
        // The aligned body as dwords (<= 65 of them: one or two stores per lane
        // instead of up to five byte stores), the unaligned head and tail bytes
        // by lanes of their own.  (A 5.4 MB mask is 22 K such runs, mean length
        // 243: the serial mask inflate's copies.)
        const uint32_t b = sm.ring[src0 & kRingMask];
        const uint32_t e = q + len, a0 = (q + 3u) & ~3u, a1 = e & ~3u;
        const uint32_t hb = (a0 < e ? a0 : e) - q;           // head bytes before the first aligned dword
        const uint32_t nd = a1 > a0 ? (a1 - a0) >> 2 : 0u;   // whole dwords
        const uint32_t ts = a1 > a0 ? a1 : a0;                // tail: [ts, e)
        const uint32_t tb = e > ts ? e - ts : 0u;
        const uint32_t w4 = b * 0x01010101u;
        for (uint32_t k = lane; k < nd; k += 64) {
          const uint32_t p = a0 + 4u * k;
          *(uint32_t *)&sm.ring[p & kRingMask] = w4;
          if (p + 4u <= want) {
            *(DG_GLOBAL uint32_t *)(out + p) = w4;
          } else {
            for (uint32_t x = 0; x < 4u; x++)
              if (p + x < want) out[p + x] = (uint8_t)b;
          }
        }
        if (lane < hb + tb) {
          const uint32_t p = lane < hb ? q + lane : ts + (lane - hb);
          sm.ring[p & kRingMask] = (uint8_t)b;
          if (p < want) out[p] = (uint8_t)b;
        }
      } else {  // every read before the writes: one LDS round trip (len <= 258)
        const float rcp = 1.0f / (float)dist;
        const bool wrap = dist < len;
        uint32_t v[5];
#pragma unroll
        for (uint32_t r = 0; r < 5; r++) {
          const uint32_t j = lane + 64u * r;
          uint32_t k = j;
          if (wrap) {  // overlapping period-`dist` copy
            const uint32_t qt = (uint32_t)((float)j * rcp);  // j / dist or one less (j < 320)
            k = j - qt * dist;
            if (k >= dist) k -= dist;
          }
          v[r] = r < rounds && j < len ? sm.ring[(src0 + k) & kRingMask] : 0u;
        }
#pragma unroll
        for (uint32_t r = 0; r < 5; r++) {
          const uint32_t j = lane + 64u * r;
          if (r < rounds && j < len) {
            sm.ring[(q + j) & kRingMask] = (uint8_t)v[r];
            if (q + j < want) out[q + j] = (uint8_t)v[r];
          }
        }
      }
      op += len;
      if (op >= want) break;
      if (consumed() > limit_bits + 64) {
        status = 2;
        break;
      }
    }
    if (consumed() > limit_bits + 64) status = 2;
  }
  if (!status && op < want) status = 2;  // stream ended before the last scanline
  stash_flush();
  __syncthreads();
  if (status && lane == 0) im.status = status;
}

// ------------------------------------------------------------ chunked inflate

// Bits [pos, pos + n) of the stream (n <= 32), LSB-first; zero past the end.
__device__ __forceinline__ uint32_t zbits(const DG_GLOBAL uint32_t *z, uint32_t zwords, uint32_t pos, uint32_t n) {
  const uint32_t w = pos >> 5, sh = pos & 31u;
  const uint64_t lo = w < zwords ? z[w] : 0u, hi = w + 1 < zwords ? z[w + 1] : 0u;
  const uint64_t v = (lo | (hi << 32)) >> sh;
  return n >= 32 ? (uint32_t)v : (uint32_t)v & ((1u << n) - 1u);
}

// Block-start candidates (k_inf_find).  A position qualifies when a
// dynamic-Huffman block header with valid, complete codes starts there: the
// checks zlib's inflate applies (HLIT <= 29, HDIST <= 29, a complete
// code-length code, a well-formed run of code lengths, an end-of-block code,
// a complete literal/length code, a complete distance code or a single
// distance code).  Two stages:
//  * inf_header_fast: header fields and the code-length code's Kraft sum, the
//    same ~100 instructions in every lane (no divergence); rejects all but
//    ~0.5% of positions;
//  * inf_header_full for the survivors: decodes the code lengths with a
//    register bit buffer and stops as soon as the literal/length or distance
//    lengths over-subscribe their code (random bits do within a few dozen
//    symbols), so a false survivor costs little.
// A false candidate only costs time downstream (the chain skips it), and every
// real dynamic block header passes, so this is a filter, not a decoder.

// bits [pos, pos + 96) from the 4 words at pos >> 5 (q[]) and pos & 31
__device__ __forceinline__ void inf_bits96(const uint32_t q[4], uint32_t sh, uint64_t &lo, uint64_t &hi) {
  const uint64_t a = (uint64_t)q[0] | ((uint64_t)q[1] << 32), b = (uint64_t)q[2] | ((uint64_t)q[3] << 32);
  lo = sh ? (a >> sh) | (b << (64 - sh)) : a;
  hi = b >> sh;
}

// Header fields + complete code-length code.  Returns the 5-bit-per-length
// histogram of the code-length code (field k = codes of length k) or 0.
__device__ __forceinline__ uint64_t inf_header_fast(uint64_t lo, uint64_t hi) {
  const uint32_t h = (uint32_t)lo & 0x1FFFFu;
  const uint32_t nlen = ((h >> 3) & 31u) + 257, ndist = ((h >> 8) & 31u) + 1, ncode = ((h >> 13) & 15u) + 4;
  const uint64_t clbits = (lo >> 17) | (hi << 47);  // bits [pos + 17, pos + 81)
  uint64_t hist = 0;
#pragma unroll
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t l = i < ncode ? (uint32_t)(clbits >> (3 * i)) & 7u : 0u;
    hist += 1ull << (5 * l);
  }
  int left = 1;
  bool bad = ((h >> 1) & 3u) != 2u || nlen > 286 || ndist > 30;
#pragma unroll
  for (uint32_t k = 1; k < 8; k++) {
    left = 2 * left - (int)((hist >> (5 * k)) & 31u);
    bad |= left < 0;
  }
  bad |= left != 0;
  return bad ? 0ull : hist | 1ull;  // bit 0 set: field 0 (length-0 count) is never read
}

// Stage 2 of the finder: the code-length code is complete (Kraft sum of its
// lengths exactly 1), in 32-bit arithmetic -- what inf_header_fast's
// per-level check amounts to (an over-subscribed level makes the sum exceed
// 1, an incomplete code leaves it short), without the 64-bit histogram
// (~6 instead of ~9 operations per length).  The header fields were stage 1's.
__device__ __forceinline__ bool inf_kraft_fast(uint64_t lo, uint64_t hi) {
  const uint32_t ncode = (((uint32_t)lo >> 13) & 15u) + 4u;
  const uint64_t clbits = (lo >> 17) | (hi << 47);  // 19 3-bit lengths from bit 0
  const uint32_t c0 = (uint32_t)clbits, c1 = (uint32_t)(clbits >> 30);  // c1: lengths 10.. at bit 0
  uint32_t k = 0;
#pragma unroll
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t l = i < 10 ? (c0 >> (3 * i)) & 7u : (c1 >> (3 * (i - 10))) & 7u;
    k += (i < ncode && l) ? 128u >> l : 0u;
  }
  return k == 128u;
}

__device__ bool inf_header_full(const DG_GLOBAL uint32_t *z, uint32_t zwords, uint32_t pos, uint64_t lo, uint64_t hi,
                                uint64_t hist) {
  const uint32_t h = (uint32_t)lo & 0x1FFFFu;
  const uint32_t nlen = ((h >> 3) & 31u) + 257, ndist = ((h >> 8) & 31u) + 1, ncode = ((h >> 13) & 15u) + 4;
  // code-length code: 3-bit lengths in c_clorder; canonical first code and
  // rank offset per length; symbols sorted by (length, symbol), 5 bits each
  uint64_t cll = 0;
  const uint64_t clbits = (lo >> 17) | (hi << 47);
  for (uint32_t i = 0; i < ncode; i++) cll |= ((clbits >> (3 * i)) & 7ull) << (3 * c_clorder[i]);
  uint32_t first[8], offs[8], cnt[8], o = 0, code = 0;
#pragma unroll
  for (uint32_t k = 1; k < 8; k++) {
    cnt[k] = (uint32_t)(hist >> (5 * k)) & 31u;
    code = (code + (k > 1 ? cnt[k - 1] : 0u)) << 1;
    first[k] = k == 1 ? 0u : code;
    offs[k] = o;
    o += cnt[k];
  }
  uint64_t sorted_lo = 0, sorted_hi = 0;  // rank r -> symbol at bits 5r (ranks 12.. in sorted_hi)
  {
    uint32_t r = 0;
    for (uint32_t k = 1; k < 8; k++)
      for (uint32_t s = 0; s < 19; s++)
        if (((uint32_t)(cll >> (3 * s)) & 7u) == k) {
          if (r < 12) sorted_lo |= (uint64_t)s << (5 * r);
          else sorted_hi |= (uint64_t)s << (5 * (r - 12));
          r++;
        }
  }
  // code lengths through a register bit buffer
  uint32_t p = pos + 17 + 3 * ncode;
  uint32_t wp = p >> 5;
  uint64_t bb = (wp < zwords ? z[wp] : 0u) >> (p & 31u);
  uint32_t nb = 32 - (p & 31u);
  wp++;
  uint32_t i = 0, prev = 0, eob = 0, dn = 0, kl = 0, kd = 0;
  const uint32_t total = nlen + ndist;
  while (i < total) {
    if (nb < 32) {
      bb |= (uint64_t)(wp < zwords ? z[wp] : 0u) << nb;
      nb += 32;
      wp++;
    }
    const uint32_t bitsv = (uint32_t)bb;
    uint32_t len = 0, rank = 0, c = 0;
#pragma unroll
    for (uint32_t k = 1; k < 8; k++) {
      c = (c << 1) | ((bitsv >> (k - 1)) & 1u);
      if (len == 0 && c - first[k] < cnt[k]) {
        len = k;
        rank = offs[k] + (c - first[k]);
      }
    }
    if (!len) return false;
    const uint32_t sym = rank < 12 ? (uint32_t)(sorted_lo >> (5 * rank)) & 31u
                                   : (uint32_t)(sorted_hi >> (5 * (rank - 12))) & 31u;
    bb >>= len;
    nb -= len;
    uint32_t v = sym, rep = 1;
    if (sym == 16) {
      if (i == 0) return false;
      v = prev;
      rep = 3 + ((uint32_t)bb & 3u);
      bb >>= 2;
      nb -= 2;
    } else if (sym == 17) {
      v = 0;
      rep = 3 + ((uint32_t)bb & 7u);
      bb >>= 3;
      nb -= 3;
    } else if (sym == 18) {
      v = 0;
      rep = 11 + ((uint32_t)bb & 127u);
      bb >>= 7;
      nb -= 7;
    }
    if (i + rep > total) return false;
    const uint32_t nl = i >= nlen ? 0u : min(rep, nlen - i), nd = rep - nl;
    if (v) {
      const uint32_t wgt = 1u << (15 - v);
      kl += nl * wgt;
      kd += nd * wgt;
      dn += nd;
      eob |= (i <= 256 && 256 < i + nl) ? 1u : 0u;
      if (kl > 32768u || kd > 32768u) return false;  // over-subscribed
    }
    prev = v;
    i += rep;
  }
  return eob && kl == 32768u && (kd == 32768u || dn == 0 || (dn == 1 && kd == 16384u));
}

// Both stages at one position (the full one only if the fast one passes).
__device__ __forceinline__ bool inf_candidate(const DG_GLOBAL uint32_t *z, uint32_t zwords, uint32_t pos) {
  const uint32_t w = pos >> 5;
  uint32_t q[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) q[k] = w + k < zwords ? z[w + k] : 0u;
  uint64_t lo, hi;
  inf_bits96(q, pos & 31u, lo, hi);
  const uint64_t hist = inf_header_fast(lo, hi);
  return hist && inf_header_full(z, zwords, pos, lo, hi, hist);
}

// One wave per chunk (but chunk 0): the first candidate block start in the
// chunk's bit range, through three filters of rising cost, each applied to
// the survivors of the last:
//  1. header fields (BFINAL = 0 -- or 1 in a second pass over a chunk the
//     first found nothing in --, BTYPE = 2, HLIT <= 29, HDIST <= 29),
//     bit-parallel: a lane tests 32 consecutive positions with a dozen 64-bit
//     shift / and operations on its two stream words, so a step covers 2048
//     positions; ~11% of random positions pass.  (Round 5: one position per
//     lane per step, ~20 instructions for 64 positions, made the finder ~60%
//     of a configs[4] batch's VALU work -- more than the decode it feeds.)
//  2. the code-length code's Kraft sum (inf_kraft_fast) on the step's
//     survivors, 64 at a time, their stream words read from the step's words
//     in LDS; ~0.4% of those pass;
//  3. inf_header_full on the Kraft survivors, once kInfStage3 of them have
//     queued (a round costs its longest lane's decode: batching more
//     positions per round scans further past the first real header;
//     template S3, option "inf_stage3").
// Every stage keeps position order, so the first position passing stage 3 is
// the first candidate of the chunk.
template <uint32_t kInfStage3>
__global__ __launch_bounds__(64) void k_inf_find(const ImageDesc *__restrict__ imgs, InfChunk *__restrict__ ch,
                                                 const WgItem *__restrict__ list) {
  __shared__ uint32_t q1pos[2048];  // stage-2 queue: the step's header-field survivors, in order
  __shared__ uint32_t qpos[128];    // stage-3 queue (Kraft survivors)
  __shared__ uint32_t win[72];      // the step's stream words W .. W + 67
  const WgItem it = list[blockIdx.x];
  InfChunk &c = ch[it.image];
  const ImageDesc &im = imgs[c.image];
  const DG_GLOBAL uint32_t *z = gp<const uint32_t>(im.png.zs);
  const uint32_t zlen = im.png.zlen, zwords = (zlen + 3) / 4;
  const uint32_t b0 = c.idx * c.span * 8u;  // a multiple of 2048 (span: a power of two >= 4096)
  const uint32_t b1 = min((c.idx + 1) * c.span * 8u, zlen * 8u);
  const uint32_t lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1ull;
  auto word = [&](uint32_t w) { return w < zwords ? z[w] : 0u; };
  uint32_t found = kInfNone;
  // stage 3 on the oldest min(qn, 64) queued positions; true when one passes
  auto stage3 = [&](uint32_t &qn) {
    __syncthreads();
    const uint32_t nb = qn < 64 ? qn : 64u;
    const uint32_t pos = qpos[lane < nb ? lane : 0];
    const bool ok = lane < nb && inf_candidate(z, zwords, pos);
    const uint64_t mo = __ballot(ok);
    if (mo) {
      found = uni(qpos[__ffsll((long long)mo) - 1]);
      return true;
    }
    const uint32_t rest = qn - nb;  // < 64
    const uint32_t keep = lane < rest ? qpos[64 + lane] : 0u;
    __syncthreads();
    if (lane < rest) qpos[lane] = keep;
    qn = rest;
    return false;
  };
  for (uint32_t bfinal = 0; bfinal < 2 && found == kInfNone; bfinal++) {
    uint32_t qn = 0;
    uint32_t nw = word((b0 >> 5) + lane), ne = lane < 4 ? word((b0 >> 5) + 64 + lane) : 0u;  // a step ahead
    for (uint32_t p = b0; p < b1 && found == kInfNone; p += 2048) {
      const uint32_t W = p >> 5;
      __syncthreads();
      win[lane] = nw;
      if (lane < 4) win[64 + lane] = ne;
      nw = word(W + 64 + lane);
      ne = lane < 4 ? word(W + 128 + lane) : 0u;
      __syncthreads();
      // stage 1: lane `lane` tests positions q .. q + 31, q = p + 32 lane
      const uint64_t A = (uint64_t)win[lane] | ((uint64_t)win[lane + 1] << 32);
      const uint32_t b1s = (uint32_t)(A >> 1), b2s = (uint32_t)(A >> 2);
      const uint32_t lit = (uint32_t)(A >> 4) & (uint32_t)(A >> 5) & (uint32_t)(A >> 6) & (uint32_t)(A >> 7);
      const uint32_t dst = (uint32_t)(A >> 9) & (uint32_t)(A >> 10) & (uint32_t)(A >> 11) & (uint32_t)(A >> 12);
      uint32_t m = (bfinal ? (uint32_t)A : ~(uint32_t)A) & ~b1s & b2s & ~lit & ~dst;
      const uint32_t q = p + 32u * lane;
      m = q >= b1 ? 0u : (b1 - q >= 32u ? m : m & ((1u << (b1 - q)) - 1u));
      // survivors into q1pos in position order: exclusive scan of the lanes' counts
      const uint32_t cnt = (uint32_t)__popc(m);
      uint32_t incl = cnt;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      const uint32_t tot = uni(__shfl(incl, 63));
      uint32_t k = incl - cnt;
      while (m) {
        q1pos[k++] = q + (uint32_t)__ffs(m) - 1u;
        m &= m - 1u;
      }
      __syncthreads();
      // stage 2, 64 survivors at a time; stage 3 once kInfStage3 queue up
      for (uint32_t r0 = 0; r0 < tot; r0 += 64) {
        const uint32_t nb = tot - r0 < 64 ? tot - r0 : 64u;
        const uint32_t pos = q1pos[r0 + (lane < nb ? lane : 0u)];
        uint32_t qw[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) qw[j] = win[(pos >> 5) - W + j];
        uint64_t lo, hi;
        inf_bits96(qw, pos & 31u, lo, hi);
        const bool pass = lane < nb && inf_kraft_fast(lo, hi);
        const uint64_t mp = __ballot(pass);
        if (pass) qpos[qn + (uint32_t)__popcll(mp & below)] = pos;
        qn += (uint32_t)__popcll(mp);
        if (qn >= kInfStage3 && stage3(qn)) break;
      }
    }
    while (found == kInfNone && qn > 0)  // the chunk's last Kraft survivors
      if (stage3(qn)) break;
  }
  if (lane == 0) c.start = found;
}

// Per-lane canonical Huffman table.  lut[1 << B] = (sym << 4) | len for codes
// of <= B bits, 0 for prefixes of longer codes and unused prefixes; the
// longer codes are walked bit-serially (puff.c's canonical decode) from length
// B + 1 with that length's first code and symbol index and the per-length
// counts held in registers, the symbol read from `sym` (sorted by length).
// k_inf_decode keeps the literal/length and distance lookups in LDS.
#define DG_LDS __attribute__((address_space(3)))
template <uint32_t B, typename LutPtr, typename SymPtr = DG_GLOBAL uint16_t *>
struct LaneTab {
  LutPtr lut;
  SymPtr sym;  // [n], by (length, symbol)
  uint32_t first1, index1;  // canonical walk state at length B + 1
  uint32_t cpk[3];          // counts of lengths B+1..15, 10 bits each, 3 per word
};

template <uint32_t B, typename LutPtr, typename SymPtr>
__device__ bool lane_build(const DG_GLOBAL uint8_t *lens, uint32_t n, LaneTab<B, LutPtr, SymPtr> &t) {
  uint32_t cnt[16];
#pragma unroll
  for (uint32_t k = 0; k < 16; k++) cnt[k] = 0;
  for (uint32_t s = 0; s < n; s++) {
    const uint32_t l = lens[s];
#pragma unroll
    for (uint32_t k = 1; k < 16; k++) cnt[k] += l == k ? 1u : 0u;
  }
  int left = 1;
  uint32_t next[16], pos[16], o = 0, code = 0, first = 0, index = 0;
#pragma unroll
  for (uint32_t k = 1; k < 16; k++) {
    left = 2 * left - (int)cnt[k];
    code = (code + (k > 1 ? cnt[k - 1] : 0u)) << 1;
    next[k] = k == 1 ? 0u : code;
    pos[k] = o;
    o += cnt[k];
    if (k == B + 1) {
      t.first1 = first;
      t.index1 = index;
    }
    index += cnt[k];
    first = (first + cnt[k]) << 1;
  }
  t.cpk[0] = t.cpk[1] = t.cpk[2] = 0;
#pragma unroll
  for (uint32_t k = B + 1; k < 16; k++) t.cpk[(k - B - 1) / 3] |= cnt[k] << (10 * ((k - B - 1) % 3));
  if (left < 0) return false;
  if (left > 0)  // incomplete: unused prefixes must read as invalid
    for (uint32_t e = 0; e < (1u << B); e++) t.lut[e] = 0;
  for (uint32_t s = 0; s < n; s++) {
    const uint32_t l = lens[s];
    if (!l) continue;
    uint32_t cd = 0, ps = 0;
#pragma unroll
    for (uint32_t k = 1; k < 16; k++)
      if (l == k) {
        cd = next[k]++;
        ps = pos[k]++;
      }
    t.sym[ps] = (uint16_t)s;
    const uint32_t rv = __builtin_bitreverse32(cd) >> (32 - l);
    if (l <= B) {
      const uint16_t e = (uint16_t)((s << 4) | l);
      for (uint32_t x = rv; x < (1u << B); x += 1u << l) t.lut[x] = e;
    } else {
      t.lut[rv & ((1u << B) - 1u)] = 0;  // long code: its B-bit prefix takes the slow path
    }
  }
  return true;
}

constexpr uint32_t kLbBuf = 8;  // Q: stream words buffered in registers per lane (default)

template <uint32_t NB = kLbBuf>
struct LaneBits {
  uint64_t bb;
  uint32_t nb, wp, zwords;  // wp: index of the next stream word to shift into bb
  uint32_t w1;              // Q = false: that word, loaded one refill ahead
  uint32_t nbuf;            // Q = true: words wp .. wp + nbuf - 1 held in buf
  uint32_t buf[NB];
};

// Q: the next kLbBuf stream words of every lane sit in registers, refilled
// for the whole wave at once (lb_top) when any lane runs low.  A per-lane
// load one word ahead (Q = false) sits in a lane-divergent branch, so the
// compiler waits for it where the branches join: every fourth symbol of a
// literal-heavy stream paid a full memory latency.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
template <uint32_t NB>
__device__ __forceinline__ void lb_fill(LaneBits<NB> &r, const DG_GLOBAL uint32_t *z) {
  static_assert(NB % 4 == 0, "whole 16-byte loads");
  const uint32_t i = r.wp;
  if (i + NB <= r.zwords) {
#pragma unroll
    for (uint32_t k = 0; k < NB; k += 4) {
      const u32x4a q = *(const DG_GLOBAL u32x4a *)(z + i + k);
      r.buf[k] = q.x;
      r.buf[k + 1] = q.y;
      r.buf[k + 2] = q.z;
      r.buf[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < NB; k++) r.buf[k] = i + k < r.zwords ? z[i + k] : 0u;
  }
  r.nbuf = NB;
}

template <bool Q, uint32_t NB>
__device__ __forceinline__ void lb_seek(LaneBits<NB> &r, const DG_GLOBAL uint32_t *z, uint32_t wp) {
  r.wp = wp;
  if (Q) {
    lb_fill(r, z);
  } else {
    r.w1 = wp < r.zwords ? z[wp] : 0u;
  }
}

// Q: at a point every lane of the wave reaches: refill all lanes' buffers
// together once any lane holds fewer words than a symbol step can take (a
// length/distance pair is at most 48 bits: two words)
template <bool Q, uint32_t NB>
__device__ __forceinline__ void lb_top(LaneBits<NB> &r, const DG_GLOBAL uint32_t *z) {
  if (Q && __ballot(r.nbuf < 3u)) lb_fill(r, z);
}

template <bool Q, uint32_t NB>
__device__ __forceinline__ void lb_refill(LaneBits<NB> &r, const DG_GLOBAL uint32_t *z) {
  if (r.nb < 32) {
    if (Q) {
      if (r.nbuf == 0) lb_fill(r, z);  // off the symbol loop (headers, stored blocks)
      r.bb |= (uint64_t)r.buf[0] << r.nb;
      r.nb += 32;
      r.wp++;
      r.nbuf--;
#pragma unroll
      for (uint32_t k = 0; k + 1 < NB; k++) r.buf[k] = r.buf[k + 1];
    } else {
      r.bb |= (uint64_t)r.w1 << r.nb;
      r.nb += 32;
      r.wp++;
      r.w1 = r.wp < r.zwords ? z[r.wp] : 0u;
    }
  }
}
template <uint32_t NB>
__device__ __forceinline__ uint32_t lb_get(LaneBits<NB> &r, uint32_t k) {
  const uint32_t v = (uint32_t)r.bb & ((1u << k) - 1u);
  r.bb >>= k;
  r.nb -= k;
  return v;
}
// consumed bit position: wp counts the word held in w1
template <uint32_t NB>
__device__ __forceinline__ uint32_t lb_pos(const LaneBits<NB> &r) { return r.wp * 32u - r.nb; }

template <uint32_t B, typename LutPtr, typename SymPtr, uint32_t NB>
__device__ __forceinline__ uint32_t lane_sym(LaneBits<NB> &r, const LaneTab<B, LutPtr, SymPtr> &t) {
  const uint32_t peek = (uint32_t)r.bb;
  const uint32_t e = t.lut[peek & ((1u << B) - 1u)];
  if (e & 15u) {
    const uint32_t l = e & 15u;
    r.bb >>= l;
    r.nb -= l;
    return e >> 4;
  }
  const uint32_t rv = __builtin_bitreverse32(peek);
  uint32_t first = t.first1, index = t.index1;
#pragma unroll
  for (uint32_t L = B + 1; L < 16; L++) {
    const uint32_t code = rv >> (32 - L);
    const uint32_t c = (t.cpk[(L - B - 1) / 3] >> (10 * ((L - B - 1) % 3))) & 1023u;
    if (code - first < c) {
      r.bb >>= L;
      r.nb -= L;
      return t.sym[index + code - first];
    }
    index += c;
    first = (first + c) << 1;
  }
  return 0xFFFFu;
}

// LDS bytes per lane: an LB-bit literal/length and a DB-bit distance lookup,
// and with SL the two symbol tables (288 + 32 entries) the canonical walk of
// longer codes reads.  Without SL those live in global memory: every code
// longer than the lookup costs the lane a dependent L2 round trip, and a
// noisy RGB stream's literal codes are mostly 8-9 bits (round 5: the
// configs[4] pool's images are literal-only deflate, ~22 KiB blocks).
// (SL: + 4 bytes, so the lanes' tables start on different banks.)
template <uint32_t LB, uint32_t DB, bool SL = false>
constexpr uint32_t inf_lds_per_lane() {
  return ((1u << LB) + (1u << DB) + (SL ? 288u + 32u + 2u : 0u)) * 2u;
}

// One lane per chunk: decode from the chunk's candidate block start until a
// block ends exactly where a later chunk's candidate starts (or the stream
// ends), writing uint16 entries: bytes, or 256 + window index for bytes that
// lie before the chunk (resolved by k_inf_resolve). WG lanes per workgroup;
// the lookups take WG * inf_lds_per_lane<LB, DB>() bytes of LDS (64 lanes,
// 9/7 bits: 80 KiB, two workgroups per CU).
template <uint32_t WG, uint32_t LB, uint32_t DB, bool Q = false, bool SL = false, uint32_t NB = kLbBuf>
__global__ __launch_bounds__(WG) void k_inf_decode(const ImageDesc *__restrict__ imgs, InfChunk *__restrict__ ch,
                                                   uint32_t nch) {
  constexpr uint32_t kInfLdsPerLane = inf_lds_per_lane<LB, DB, SL>();
  const uint32_t gi = blockIdx.x * WG + threadIdx.x;
  if (gi >= nch) return;
  InfChunk &c = ch[gi];
  c.len = 0;
  c.status = 0;
  const ImageDesc &im = imgs[c.image];
  const PngDesc &pd = im.png;
  const uint32_t n = pd.nchunks;
  c.stop = n;
  if (c.start == kInfNone) return;
  const InfChunk *img_ch = ch + pd.chunk0;
  const DG_GLOBAL uint32_t *z = gp<const uint32_t>(pd.zs);
  DG_GLOBAL uint16_t *out = gp<uint16_t>(c.out);
  DG_GLOBAL uint8_t *tb = gp<uint8_t>(c.tab);
  DG_GLOBAL uint8_t *lens = tb + 3584;
  // LDS: per lane a 9-bit literal/length and a 7-bit distance lookup
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  DG_LDS uint16_t *lds = (DG_LDS uint16_t *)(DG_LDS uint8_t *)smem_raw + threadIdx.x * kInfLdsPerLane / 2;
  using SymP = typename std::conditional<SL, DG_LDS uint16_t *, DG_GLOBAL uint16_t *>::type;
  SymP lsym, dsym;
  if constexpr (SL) {
    lsym = lds + (1u << LB) + (1u << DB);
    dsym = lsym + 288;
  } else {
    lsym = (DG_GLOBAL uint16_t *)(tb + 2624);
    dsym = (DG_GLOBAL uint16_t *)(tb + 3264);
  }
  LaneTab<LB, DG_LDS uint16_t *, SymP> tl{lds, lsym, 0, 0, {0, 0, 0}};
  LaneTab<DB, DG_LDS uint16_t *, SymP> td{lds + (1u << LB), dsym, 0, 0, {0, 0, 0}};
  LaneTab<6, DG_GLOBAL uint16_t *> tc{(DG_GLOBAL uint16_t *)(tb + 3328), (DG_GLOBAL uint16_t *)(tb + 3520), 0, 0,
                                      {0, 0, 0}};
  const uint32_t zbits_total = pd.zlen * 8u;
  LaneBits<NB> r;
  r.zwords = (pd.zlen + 3) / 4;
  {
    const uint32_t p = c.start;
    r.bb = 0;
    r.nb = 0;
    lb_seek<Q>(r, z, p >> 5);
    lb_refill<Q>(r, z);
    lb_get(r, p & 31u);
  }
  const uint32_t cap = c.cap;
  const bool first_chunk = c.idx == 0;
  uint32_t q = 0;  // entries produced
  uint32_t nxt = c.idx + 1;
  uint32_t status = 0;
  for (;;) {
    // block boundary: stop if a later chunk starts exactly here
    const uint32_t bp = lb_pos(r);
    while (nxt < n && (img_ch[nxt].start == kInfNone || img_ch[nxt].start < bp)) nxt++;
    if (nxt < n && img_ch[nxt].start == bp && bp != c.start) {
      c.stop = nxt;
      break;
    }
    if (bp > zbits_total) {
      status = 1;
      break;
    }
    lb_refill<Q>(r, z);
    const uint32_t last = lb_get(r, 1), type = lb_get(r, 2);
    if (type == 3) {
      status = 1;
      break;
    }
    if (type == 0) {
      lb_get(r, r.nb & 7u);
      lb_refill<Q>(r, z);
      const uint32_t len = lb_get(r, 16), nlen = lb_get(r, 16);
      if ((len ^ 0xFFFFu) != nlen) {
        status = 1;
        break;
      }
      const uint32_t bpos = lb_pos(r) / 8u;
      if (bpos + len > pd.zlen || q + len > cap) {
        status = bpos + len > pd.zlen ? 1u : 2u;
        break;
      }
      const DG_GLOBAL uint8_t *zb = (const DG_GLOBAL uint8_t *)z;
      for (uint32_t j = 0; j < len; j++) out[q + j] = zb[bpos + j];
      q += len;
      const uint32_t np = (bpos + len) * 8u;
      r.bb = 0;
      r.nb = 0;
      lb_seek<Q>(r, z, np >> 5);
      lb_refill<Q>(r, z);
      lb_get(r, np & 31u);
      if (last) break;
      continue;
    }
    if (type == 1) {
      for (uint32_t s = 0; s < 320; s++) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
      lane_build(lens, 288, tl);
      lane_build(lens + 288, 30, td);
    } else {
      lb_refill<Q>(r, z);
      const uint32_t nlen = lb_get(r, 5) + 257, ndist = lb_get(r, 5) + 1, ncode = lb_get(r, 4) + 4;
      if (nlen > 286 || ndist > 30) {
        status = 1;
        break;
      }
      for (uint32_t s = 0; s < 19; s++) lens[s] = 0;
      for (uint32_t i = 0; i < ncode; i++) {
        lb_refill<Q>(r, z);
        lens[c_clorder[i]] = (uint8_t)lb_get(r, 3);
      }
      if (!lane_build(lens, 19, tc)) {
        status = 1;
        break;
      }
      uint32_t i = 0, prev = 0;
      const uint32_t total = nlen + ndist;
      while (i < total && !status) {
        lb_refill<Q>(r, z);
        const uint32_t s = lane_sym(r, tc);
        uint32_t v = s, rep = 1;
        if (s < 16) {
        } else if (s == 16 && i > 0) {
          v = prev;
          rep = 3 + lb_get(r, 2);
        } else if (s == 17) {
          v = 0;
          rep = 3 + lb_get(r, 3);
        } else if (s == 18) {
          v = 0;
          rep = 11 + lb_get(r, 7);
        } else {
          status = 1;
          break;
        }
        if (i + rep > total) {
          status = 1;
          break;
        }
        // litlen lengths at [0, nlen), distance lengths at [288, 288 + ndist)
        for (uint32_t k = 0; k < rep; k++, i++) lens[i < nlen ? i : 288 + (i - nlen)] = (uint8_t)v;
        prev = v;
      }
      if (status) break;
      if (lens[256] == 0 || !lane_build(lens, nlen, tl) || !lane_build(lens + 288, ndist, td)) {
        status = 1;
        break;
      }
    }
    // symbols of the block
    for (;;) {
      lb_top<Q>(r, z);
      lb_refill<Q>(r, z);
      const uint32_t s = lane_sym(r, tl);
      if (s < 256) {
        if (q >= cap) {
          status = 2;
          break;
        }
        out[q++] = (uint16_t)s;
        continue;
      }
      if (s == 256) break;
      if (s > 285) {
        status = 1;
        break;
      }
      const uint32_t lx = c_lenx[s - 257];
      const uint32_t len = (lx & 0xFFFFu) + lb_get(r, lx >> 16);
      lb_refill<Q>(r, z);
      const uint32_t ds = lane_sym(r, td);
      if (ds >= 30) {
        status = 1;
        break;
      }
      lb_refill<Q>(r, z);
      const uint32_t dx = c_distx[ds];
      const uint32_t dist = (dx & 0xFFFFu) + lb_get(r, dx >> 16);
      if (q + len > cap) {
        status = 2;
        break;
      }
      if (dist > q && first_chunk) {
        status = 1;
        break;
      }
      // sources lie before q: entries of this chunk, or markers into the
      // window before it (256 + 32768 + (src - 0) for src < 0)
      int32_t src = (int32_t)q - (int32_t)dist;
      const int32_t s0 = src;
      uint32_t j = 0;
      for (; j + 4 <= len; j += 4) {
        uint16_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int32_t sp = s0 + (int32_t)((dist >= len) ? (j + u) : ((j + u) % dist));
          v[u] = sp >= 0 ? out[sp] : (uint16_t)(256 + 32768 + sp);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) out[q + j + u] = v[u];
      }
      for (; j < len; j++) {
        const int32_t sp = s0 + (int32_t)((dist >= len) ? j : (j % dist));
        out[q + j] = sp >= 0 ? out[sp] : (uint16_t)(256 + 32768 + sp);
      }
      (void)src;
      q += len;
    }
    if (status) break;
    if (last) break;
  }
  c.len = q;
  c.status = status;
}

// One workgroup per chunked image: walk the chain of chunks the decode made
// consistent, resolving each chunk's entries into the scanline buffer in
// order (a chunk's markers read the 32 KiB written just before it).
__global__ __launch_bounds__(1024) void k_inf_resolve(ImageDesc *__restrict__ imgs, const InfChunk *__restrict__ ch,
                                                      const WgItem *__restrict__ list) {
  const WgItem it = list[blockIdx.x];
  ImageDesc &im = imgs[it.image];
  PngDesc &pd = im.png;
  const uint32_t want = pd.rawlen;
  DG_GLOBAL uint8_t *raw = gp<uint8_t>(pd.raw);
  const InfChunk *c0 = ch + pd.chunk0;
  uint32_t k = 0, P = 0;
  bool bad = false;
  while (k < pd.nchunks && P < want) {
    const InfChunk &c = c0[k];
    if (c.status || c.start == kInfNone) {
      bad = true;
      break;
    }
    const DG_GLOBAL uint16_t *e = gp<const uint16_t>(c.out);
    const uint32_t n = min(c.len, want - P);
    uint32_t oob = 0;
    // 8 entries per thread per round, every load issued before any store: a
    // marker reads bytes before P (earlier chunks, already fenced), never this
    // chunk's, so nothing orders the loads after the stores
    constexpr uint32_t U = 8;
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += 1024 * U) {
      uint32_t v[U];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint32_t i = i0 + 1024 * u;
        v[u] = i < n ? e[i] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        if (v[u] >= 256) {
          const int64_t sp = (int64_t)P - 32768 + (int64_t)(v[u] - 256);
          oob |= sp < 0 ? 1u : 0u;
          v[u] = sp < 0 ? 0u : (uint32_t)raw[sp];
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint32_t i = i0 + 1024 * u;
        if (i < n) raw[P + i] = (uint8_t)v[u];
      }
    }
    if (__syncthreads_or(oob)) {
      bad = true;
      break;
    }
    // a workgroup-scope fence + barrier makes this chunk's bytes visible to
    // the next chunk's marker loads (every thread is on this CU); the
    // device-scope __threadfence used before wrote the L2 back on every chunk
    // (k_inf_resolve 18 -> 5 ms per batch without it)
    __syncthreads();
    P += n;
    if (c.stop <= k) {  // cannot go backwards
      bad = true;
      break;
    }
    k = c.stop;
  }
  if (P < want) bad = true;
  if (bad && threadIdx.x == 0) pd.serial = 1;
}

// ------------------------------------------------------------ unfilter

// One wave per band of 64 rows, lane l owning row y0 + l,
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

// The band's raw bytes are staged through LDS in tiles of kUfTile filter
// units x 64 rows (coalesced loads; the diagonal then reads and writes LDS
// only), three tiles in flight: lane 0 enters tile k while lanes 1..63 finish
// tile k-1; tile k-2 is complete, is stored to HBM, and its buffer receives
// tile k+1.  Each lane takes kUfU units per step (lane l at step t owns units
// kUfU*(t-l) ..), so one shuffle round trip serves kUfU units.
// kUfU is a template parameter (option uf_units, 1 or 2; default 2).
// LDS of one worker: 3 tiles of 64 rows plus 3 previous-band rows, each
// kUfTile * bpp + 4 bytes (dword misalignment; an odd number of words, so
// lane rows fall on distinct banks).  Sized for the batch's widest filter
// unit (dynamic LDS), so batches of 1-3-byte units run more workers per CU.
__host__ __device__ constexpr uint32_t uf_pitch(uint32_t bpp, uint32_t u) { return 64 * u * bpp + 4; }
__host__ __device__ constexpr uint32_t uf_smem_bytes(uint32_t bpp, uint32_t u) { return (3 * 64 + 3) * uf_pitch(bpp, u); }
struct UnfilterSmem {
  uint8_t *base;
  uint32_t pitch;
  __device__ __forceinline__ uint8_t *tile(uint32_t k, uint32_t r) const { return base + ((k % 3) * 64 + r) * pitch; }
  __device__ __forceinline__ uint8_t *prow(uint32_t k) const { return base + (192 + k % 3) * pitch; }
};

template <uint32_t BPP>
__device__ __forceinline__ uint32_t unfilter_unit(uint32_t f, uint32_t rawv, uint32_t a, uint32_t b, uint32_t c) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < BPP; k++) {
    const uint32_t sh = 8 * k;
    const uint32_t ak = (a >> sh) & 0xFFu, bk = (b >> sh) & 0xFFu, ck = (c >> sh) & 0xFFu;
    const uint32_t pr = f == 0 ? 0u : f == 1 ? ak : f == 2 ? bk : f == 3 ? (ak + bk) >> 1 : paeth_b(ak, bk, ck);
    v |= ((((rawv >> sh) & 0xFFu) + pr) & 0xFFu) << sh;
  }
  return v;
}

// Progress of a band (one 64-row band of one plane): tiles of its rows stored
// to HBM, kUfDone when the band is finished or skipped.  The next band of the
// plane reads this band's last row tile by tile as it becomes available, so
// consecutive bands run as a pipeline on different CUs, about three tiles
// apart.
constexpr uint32_t kUfDone = 0xFFFFFFFFu;

// (every lane stores the same value: no lane-0 branch in the waves' control
// flow, which the compiler's loop structurizer mishandled here)
__device__ __forceinline__ void uf_publish(DG_GLOBAL uint32_t *flag, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's tile stores before the flag
  __hip_atomic_store((uint32_t *)flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until *flag >= need.  False after ~1 s of s_memrealtime (100 MHz) --
// a producer that never comes, or one starved by other work on the device
// (ranks sharing a GPU): the caller then returns the image
// DG_ERR_UNSUPPORTED, so the CPU decodes it, rather than hang the device.
// `force` (test switch kDbgForceUfTimeout) times out at once.
__device__ __forceinline__ bool uf_wait(const DG_GLOBAL uint32_t *flag, uint32_t need, bool force) {
  if (force) return false;
  uint64_t t0 = 0;
  for (;;) {
    const uint32_t v = uni(__hip_atomic_load((uint32_t *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v >= need) break;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (!t0) t0 = now;
    if (now - t0 > 100000000ull) return false;
    __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// Rows [y0, y0 + 64) of one filtered plane (the image, or one Adam7 pass) of
// H rows of 1 + rb bytes at raw_a -> rows of rb bytes at stride us at unf_a.
// `pred` is the previous band's progress flag (null for the first band).
template <uint32_t BPP, uint32_t kUfU>
__device__ void unfilter_band(const UnfilterSmem &sm, ImageDesc &im, uint64_t raw_a, uint64_t unf_a, uint32_t rb,
                              uint32_t us, uint32_t H, uint32_t y0, DG_GLOBAL uint32_t *self,
                              const DG_GLOBAL uint32_t *pred, bool force_timeout) {
  constexpr uint32_t kUfTile = 64 * kUfU;
  const uint32_t lane = threadIdx.x;
  const uint32_t units = rb / BPP;  // BPP == 1 covers sub-byte samples (filter unit = 1 byte)
  const uint32_t tb = kUfTile * BPP;
  const uint32_t ntiles = (units + kUfTile - 1) / kUfTile;
  const DG_GLOBAL uint8_t *raw = gp<const uint8_t>(raw_a);
  DG_GLOBAL uint8_t *unf = gp<uint8_t>(unf_a);
  int bad = 0;    // a filter type byte > 4: the stream is corrupt
  int stall = 0;  // the previous band's wait timed out: valid data, not decoded here
  {
    const uint32_t nrows = H - y0 < 64 ? H - y0 : 64;
    const bool active = lane < nrows;
    uint32_t f = active ? raw[(size_t)(y0 + lane) * (rb + 1)] : 0u;
    if (f > 4) {
      bad = 1;
      f = 0;
    }
    // Tiles arrive by LDS-DMA (global_load_lds_dword, no VGPR round trip,
    // retired by the vmcnt wait of the next tile boundary's barrier).  Raw
    // rows are not dword aligned: each row lands whole-word aligned and the
    // row's first byte sits at roff (0..3) in its LDS row.
    const uint64_t rbase = raw_a + (uint64_t)y0 * (rb + 1) + 1;
    auto roff = [&](uint32_t r) { return (uint32_t)((rbase + (uint64_t)r * (rb + 1)) & 3u); };
    auto load_tile = [&](uint32_t k) {
      const uint32_t b0 = k * tb, nb = rb - b0 < tb ? rb - b0 : tb;
      for (uint32_t r = 0; r < nrows; r++) {
        const uint64_t a = rbase + (uint64_t)r * (rb + 1) + b0, a4 = a & ~(uint64_t)3;
        const uint32_t nw = (uint32_t)((a - a4 + nb + 3) / 4);
        for (uint32_t w0 = 0; w0 < nw; w0 += 64)
          if (w0 + lane < nw)
            __builtin_amdgcn_global_load_lds((const DG_GLOBAL void *)(uintptr_t)(a4 + 4ull * (w0 + lane)),
                                             (__attribute__((address_space(3))) void *)(sm.tile(k, r) + 4 * w0), 4, 0, 0);
      }
      if (y0) {
        if (!stall && !uf_wait(pred, k + 1, force_timeout)) stall = 1;
        const uint64_t a = unf_a + (uint64_t)(y0 - 1) * us + b0;
        const uint32_t nw = (nb + 3) / 4;
        for (uint32_t w0 = 0; w0 < nw; w0 += 64)
          if (w0 + lane < nw)
            __builtin_amdgcn_global_load_lds((const DG_GLOBAL void *)(uintptr_t)(a + 4ull * (w0 + lane)),
                                             (__attribute__((address_space(3))) void *)(sm.prow(k) + 4 * w0), 4,
                                             0, 0);
      } else {
        for (uint32_t c = lane; c < nb; c += 64) sm.prow(k)[c] = 0;
      }
    };
    auto store_tile = [&](uint32_t k) {
      const uint32_t b0 = k * tb, nb = rb - b0 < tb ? rb - b0 : tb;
      const uint32_t nw = (nb + 3) / 4;  // whole words: the tail lands in the row's stride padding
      for (uint32_t r = 0; r < nrows; r++) {
        DG_GLOBAL uint32_t *dst = (DG_GLOBAL uint32_t *)(unf + (size_t)(y0 + r) * us + b0);
        const uint32_t o = roff(r);
        const uint32_t *src = (const uint32_t *)sm.tile(k, r);
        for (uint32_t c = lane; c < nw; c += 64) dst[c] = __builtin_amdgcn_alignbyte(src[c + 1], src[c], o);
      }
    };
    const uint32_t myoff = roff(lane < nrows ? lane : 0);
    load_tile(0);
    if (ntiles > 1) load_tile(1);
    uint32_t stored = 0;  // tiles [0, stored) are in HBM
    __syncthreads();
    uint32_t prev[kUfU], prev2 = 0;  // this lane's results of step t-1; last unit of step t-2
#pragma unroll
    for (uint32_t j = 0; j < kUfU; j++) prev[j] = 0;
    const uint32_t nsteps = (units + kUfU - 1) / kUfU + 63;
    for (uint32_t t = 0; t < nsteps; t++) {
      if ((t & 63) == 0 && t > 0) {
        const uint32_t k = t / 64;  // lane 0 enters tile k; tile k-2 is complete
        if (k >= 2) {
          store_tile(k - 2);
          stored = k - 1;
          uf_publish(self, stored);
        }
        if (k + 1 < ntiles) load_tile(k + 1);
        __syncthreads();
      }
      const int32_t x0 = (int32_t)(kUfU * t) - (int32_t)(kUfU * lane);
      // this step's raw samples (independent of the shuffles below)
      uint32_t rawv[kUfU];
      uint8_t *Tp[kUfU];
#pragma unroll
      for (uint32_t j = 0; j < kUfU; j++) {
        const int32_t x = x0 + (int32_t)j;
        const bool ok = active && x >= 0 && (uint32_t)x < units;
        const uint32_t xx = ok ? (uint32_t)x : 0u;
        Tp[j] = sm.tile(xx / kUfTile, lane) + myoff + (xx % kUfTile) * BPP;
        uint32_t v = 0;
#pragma unroll
        for (uint32_t k = 0; k < BPP; k++) v |= (uint32_t)Tp[j][k] << (8 * k);
        rawv[j] = v;
      }
      // row above: lane l-1's units of step t-1; above-left of unit 0: its last unit of step t-2
      uint32_t up[kUfU];
#pragma unroll
      for (uint32_t j = 0; j < kUfU; j++) up[j] = shfl_up1(prev[j]);
      uint32_t ul0 = shfl_up1(prev2);
      if (lane == 0 && x0 >= 0 && (uint32_t)x0 < units) {  // the previous band's last row
#pragma unroll
        for (uint32_t j = 0; j < kUfU; j++) {
          const uint32_t x = (uint32_t)x0 + j < units ? (uint32_t)x0 + j : (uint32_t)x0;
          const uint8_t *pr = sm.prow(x / kUfTile) + (x % kUfTile) * BPP;
          uint32_t v = 0;
#pragma unroll
          for (uint32_t k = 0; k < BPP; k++) v |= (uint32_t)pr[k] << (8 * k);
          up[j] = v;
        }
        ul0 = 0;
        if (x0 > 0) {
          const uint32_t x = (uint32_t)x0 - 1;
          const uint8_t *pr = sm.prow(x / kUfTile) + (x % kUfTile) * BPP;
#pragma unroll
          for (uint32_t k = 0; k < BPP; k++) ul0 |= (uint32_t)pr[k] << (8 * k);
        }
      }
      uint32_t cur[kUfU];
      uint32_t left = x0 > 0 ? prev[kUfU - 1] : 0u, ul = x0 > 0 ? ul0 : 0u;
#pragma unroll
      for (uint32_t j = 0; j < kUfU; j++) {
        const int32_t x = x0 + (int32_t)j;
        const bool ok = active && x >= 0 && (uint32_t)x < units;
        const uint32_t v = unfilter_unit<BPP>(f, rawv[j], left, up[j], ul);
        cur[j] = ok ? v : 0u;
        if (ok) {
#pragma unroll
          for (uint32_t k = 0; k < BPP; k++) Tp[j][k] = (uint8_t)(v >> (8 * k));
        }
        left = v;
        ul = up[j];
      }
      prev2 = prev[kUfU - 1];
#pragma unroll
      for (uint32_t j = 0; j < kUfU; j++) prev[j] = cur[j];
    }
    __syncthreads();
    for (uint32_t k = stored; k < ntiles; k++) store_tile(k);
  }
  const bool any_bad = __ballot(bad) != 0, any_stall = __ballot(stall) != 0;
  if (lane == 0) {
    if (any_bad)
      im.status = 2;  // DG_ERR_CORRUPT: drop the sample, as image::ImageError does
    else if (any_stall)
      atomicCAS((int *)&im.status, 0, 1);  // DG_ERR_UNSUPPORTED (CORRUPT from another band wins)
  }
}

// Persistent workers over the batch's bands: a worker takes the next band in
// ticket order (bands of all planes round-robin, band 0 of every plane first),
// so a band's predecessor was always taken earlier by a running worker and
// every wait ends (no dependence on which workgroups are resident).
template <uint32_t U>
__global__ __launch_bounds__(64) void k_png_unfilter(ImageDesc *__restrict__ imgs, const WgItem *__restrict__ tasks,
                                                     uint32_t ntasks, uint32_t *__restrict__ flags_,
                                                     uint32_t *__restrict__ ticket, uint32_t dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t uf_smem[];  // uf_smem_bytes(batch's widest unit, U)
  __shared__ uint32_t s_ticket;
  // a band is a serial wavefront on its image's critical path, as the serial
  // inflate (k_png_inflate): issue priority over the other batches' waves
  __builtin_amdgcn_s_setprio(2);
  DG_GLOBAL uint32_t *flags = gp<uint32_t>((uint64_t)(uintptr_t)flags_);
  for (;;) {
    if (threadIdx.x == 0) s_ticket = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t t = s_ticket;
    __syncthreads();
    if (t >= ntasks) break;
    const WgItem it = tasks[t];
    ImageDesc &im = imgs[it.image];
    const PngDesc &pd = im.png;
    const uint32_t pass = it.item0 >> 24, band = it.item0 & 0xFFFFFFu;
    uint64_t ra = pd.raw, ua = pd.unf;
    uint32_t rb = pd.rowbytes, us = pd.ustride, H = im.height, foff = 0;
    if (pd.interlace) {  // Adam7 pass: a sub-image of its own (PNG spec 8.2)
      const uint32_t spp = pd.ctype == 2 ? 3u : pd.ctype == 4 ? 2u : pd.ctype == 6 ? 4u : 1u;
      const A7Pass a = png_adam7(im.width, im.height, spp * pd.depth, pass);
      ra += a.raw_off;
      ua += a.unf_off;
      rb = a.rb;
      us = a.us;
      H = a.ph;
      for (uint32_t q = 0; q < pass; q++) {
        uint32_t pw, ph;
        png_adam7_pass(im.width, im.height, q, pw, ph);
        if (pw && ph) foff += (ph + 63) / 64;
      }
    }
    DG_GLOBAL uint32_t *self = flags + pd.uf_flag0 + foff + band;
    const DG_GLOBAL uint32_t *pred = band ? self - 1 : nullptr;
    // test switch (debug_flags bit 18): band 1 of every plane times out on its first wait
    const bool force = (dbg & 1u) && band == 1;
    if (!uni(im.status)) {  // (an image whose inflate failed has nothing to unfilter)
      const UnfilterSmem sm{uf_smem, uf_pitch(pd.bpp <= 4 ? pd.bpp : 4, U)};
      switch (pd.bpp) {
        case 1: unfilter_band<1, U>(sm, im, ra, ua, rb, us, H, band * 64, self, pred, force); break;
        case 2: unfilter_band<2, U>(sm, im, ra, ua, rb, us, H, band * 64, self, pred, force); break;
        case 3: unfilter_band<3, U>(sm, im, ra, ua, rb, us, H, band * 64, self, pred, force); break;
        default: unfilter_band<4, U>(sm, im, ra, ua, rb, us, H, band * 64, self, pred, force); break;
      }
    }
    uf_publish(self, kUfDone);  // the next band's tiles read this band's last row from HBM
  }
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
  const uint32_t y = idx / W, xo = idx - y * W;
  const uint32_t C = im.dec_c;
  DG_GLOBAL uint8_t *o = gp<uint8_t>(im.pix) + (size_t)y * im.pix_stride + (size_t)xo * C;
  const DG_GLOBAL uint8_t *r;
  uint32_t x = xo;  // sample index in the source row
  if (pd.interlace) {  // Adam7: the pass holding (x, y) and the pixel's place in it
    const uint32_t spp = pd.ctype == 2 ? 3u : pd.ctype == 4 ? 2u : pd.ctype == 6 ? 4u : 1u;
    const uint32_t xm = xo & 7u, ym = y & 7u;
    const uint32_t p = (ym & 1u) ? 6u : (xm & 1u) ? 5u : (ym & 2u) ? 4u : (xm & 2u) ? 3u : (ym & 4u) ? 2u
                     : (xm & 4u) ? 1u : 0u;
    const A7Pass a = png_adam7(W, im.height, spp * pd.depth, p);
    x = (xo - png_a7(p, 0)) / png_a7(p, 2);
    r = gp<const uint8_t>(pd.unf) + a.unf_off + (size_t)((y - png_a7(p, 1)) / png_a7(p, 3)) * a.us;
  } else {
    r = gp<const uint8_t>(pd.unf) + (size_t)y * pd.ustride;
  }
  const uint32_t dp = pd.depth;
  if (dp == 8 && !pd.has_trns && pd.ctype != 3) {  // de-interlace only: copy the pixel
    for (uint32_t c = 0; c < C; c++) o[c] = r[(size_t)x * C + c];
  } else if (pd.ctype == 0 || pd.ctype == 3) {
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
void launch_png_inflate(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, int mode,
                        BatchFlags *flags, uint32_t ncu) {
  static bool attr = false;  // > 64 KiB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_png_inflate, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(InflateSmem));
    attr = true;
  }
  const uint32_t grid = mode == 1 ? std::min<uint32_t>(nwg, ncu) : nwg;
  if (grid)
    hipLaunchKernelGGL(k_png_inflate, dim3(grid), dim3(64), sizeof(InflateSmem), st, imgs, list, nwg, mode, flags);
}
void launch_inf_find(hipStream_t st, const ImageDesc *imgs, InfChunk *ch, const WgItem *list, uint32_t nwg,
                     uint32_t stage3) {
  if (!nwg) return;
  switch (stage3) {
    case 8: hipLaunchKernelGGL(k_inf_find<8>, dim3(nwg), dim3(64), 0, st, imgs, ch, list); break;
    case 16: hipLaunchKernelGGL(k_inf_find<16>, dim3(nwg), dim3(64), 0, st, imgs, ch, list); break;
    case 64: hipLaunchKernelGGL(k_inf_find<64>, dim3(nwg), dim3(64), 0, st, imgs, ch, list); break;
    default: hipLaunchKernelGGL(k_inf_find<32>, dim3(nwg), dim3(64), 0, st, imgs, ch, list); break;
  }
}
template <uint32_t WG, uint32_t LB, uint32_t DB, bool Q = false, bool SL = false, uint32_t NB = kLbBuf>
static void launch_inf_decode_t(hipStream_t st, const ImageDesc *imgs, InfChunk *ch, uint32_t nch) {
  constexpr uint32_t lds = WG * inf_lds_per_lane<LB, DB, SL>();
  static bool attr = false;  // > 64 KiB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_inf_decode<WG, LB, DB, Q, SL, NB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (nch)
    hipLaunchKernelGGL((k_inf_decode<WG, LB, DB, Q, SL, NB>), dim3((nch + WG - 1) / WG), dim3(WG), lds, st, imgs, ch,
                       nch);
}
// variant: 64-lane workgroups with 0 = 9/7-bit lookups (80 KiB, 2 per CU);
// 1 = 8/6 bits (40 KiB, 4 per CU); 2 = 7/6 bits (24 KiB, 6 per CU);
// 3 = 7/5 bits (20 KiB, 8 per CU); 4 = 6/5 bits (12 KiB); 5 = 6/4 bits
// (10 KiB); 6 / 7 = 2 / 1 with the wave-batched register stream buffer
// (lb_top / lb_refill<true>). 32-lane workgroups measured no faster
// than 64-lane ones of the same LDS (profiles/r03/infdec)
void launch_inf_decode(hipStream_t st, const ImageDesc *imgs, InfChunk *ch, uint32_t nch, uint32_t variant) {
  switch (variant) {
    case 1: launch_inf_decode_t<64, 8, 6>(st, imgs, ch, nch); break;
    case 2: launch_inf_decode_t<64, 7, 6>(st, imgs, ch, nch); break;
    case 3: launch_inf_decode_t<64, 7, 5>(st, imgs, ch, nch); break;
    case 4: launch_inf_decode_t<64, 6, 5>(st, imgs, ch, nch); break;
    case 5: launch_inf_decode_t<64, 6, 4>(st, imgs, ch, nch); break;
    case 6: launch_inf_decode_t<64, 7, 6, true>(st, imgs, ch, nch); break;   // 2 + register buffer
    case 7: launch_inf_decode_t<64, 8, 6, true>(st, imgs, ch, nch); break;   // 1 + register buffer
    // symbol tables in LDS (SL): 7/6 bits 64 KiB per wave, 6/5 52 KiB, 8/6 96 KiB; 12 / 13 = 8 / 9 with the
    // register buffer (neither the walk's symbol read nor a stream load on a lane's per-symbol path)
    case 8: launch_inf_decode_t<64, 7, 6, false, true>(st, imgs, ch, nch); break;
    case 9: launch_inf_decode_t<64, 6, 5, false, true>(st, imgs, ch, nch); break;
    case 11: launch_inf_decode_t<64, 8, 6, false, true>(st, imgs, ch, nch); break;
    case 12: launch_inf_decode_t<64, 7, 6, true, true>(st, imgs, ch, nch); break;
    case 13: launch_inf_decode_t<64, 6, 5, true, true>(st, imgs, ch, nch); break;
    case 14: launch_inf_decode_t<64, 9, 7, true>(st, imgs, ch, nch); break;
    case 15: launch_inf_decode_t<64, 8, 6, true, true>(st, imgs, ch, nch); break;
    case 16: launch_inf_decode_t<64, 7, 5, true>(st, imgs, ch, nch); break;   // 3 + register buffer
    case 17: launch_inf_decode_t<64, 7, 4>(st, imgs, ch, nch); break;         // 18 KiB
    case 18: launch_inf_decode_t<64, 8, 5>(st, imgs, ch, nch); break;         // 36 KiB
    case 19: launch_inf_decode_t<64, 8, 4>(st, imgs, ch, nch); break;         // 34 KiB
    case 20: launch_inf_decode_t<64, 7, 4, true>(st, imgs, ch, nch); break;   // 17 + register buffer
    case 21: launch_inf_decode_t<64, 6, 5, true>(st, imgs, ch, nch); break;   // 4 + register buffer
    case 22: launch_inf_decode_t<64, 6, 4, true>(st, imgs, ch, nch); break;   // 5 + register buffer
    case 23: launch_inf_decode_t<64, 7, 5, true, false, 4>(st, imgs, ch, nch); break;   // 16, 4 words
    case 24: launch_inf_decode_t<64, 7, 5, true, false, 12>(st, imgs, ch, nch); break;  // 16, 12 words
    case 25: launch_inf_decode_t<64, 7, 5, true, false, 16>(st, imgs, ch, nch); break;  // 16, 16 words
    case 26: launch_inf_decode_t<64, 7, 5, true, false, 24>(st, imgs, ch, nch); break;  // 16, 24 words
    case 27: launch_inf_decode_t<64, 7, 5, true, false, 32>(st, imgs, ch, nch); break;  // 16, 32 words
    case 28: launch_inf_decode_t<64, 7, 4, true, false, 16>(st, imgs, ch, nch); break;  // 20, 16 words
    default: launch_inf_decode_t<64, 9, 7>(st, imgs, ch, nch); break;
  }
}
void launch_inf_resolve(hipStream_t st, ImageDesc *imgs, const InfChunk *ch, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_inf_resolve, dim3(nwg), dim3(1024), 0, st, imgs, ch, list);
}
template <uint32_t U>
static void launch_png_unfilter_t(uint32_t max_per_cu, hipStream_t st, ImageDesc *imgs, const WgItem *tasks, uint32_t ntasks,
                                  uint32_t *flags, uint32_t ncu, uint32_t maxbpp, uint32_t dbg) {
  // flags: ntasks progress words + the ticket counter, zeroed by the caller
  static bool attr = false;  // > 64 KiB of dynamic LDS
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_png_unfilter<U>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)uf_smem_bytes(4, U));
    attr = true;
  }
  const uint32_t bpp = maxbpp < 1 ? 1u : maxbpp > 4 ? 4u : maxbpp, lds = uf_smem_bytes(bpp, U);
  uint32_t per_cu = std::max<uint32_t>(1u, (160u * 1024u - 64u) / (lds + 64u));  // workers resident per CU
  if (max_per_cu && per_cu > max_per_cu) per_cu = max_per_cu;
  const uint32_t g = std::min(ntasks, ncu * per_cu);
  if (g)
    hipLaunchKernelGGL(k_png_unfilter<U>, dim3(g), dim3(64), lds, st, imgs, tasks, ntasks, flags, flags + ntasks, dbg);
}
// units: filter units per lane per diagonal step (tiles of 64 * units columns;
// 1 halves the LDS per worker, 2 halves the shuffle round trips per unit)
void launch_png_unfilter(hipStream_t st, ImageDesc *imgs, const WgItem *tasks, uint32_t ntasks, uint32_t *flags,
                         uint32_t ncu, uint32_t maxbpp, uint32_t dbg, uint32_t units, uint32_t max_per_cu) {
  if (units == 1)
    launch_png_unfilter_t<1>(max_per_cu, st, imgs, tasks, ntasks, flags, ncu, maxbpp, dbg);
  else
    launch_png_unfilter_t<2>(max_per_cu, st, imgs, tasks, ntasks, flags, ncu, maxbpp, dbg);
}
void launch_png_expand(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg) {
  if (nwg) hipLaunchKernelGGL(k_png_expand, dim3(nwg), dim3(256), 0, st, imgs, list);
}
void launch_alpha(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int point) {
  if (nwg) hipLaunchKernelGGL(k_alpha, dim3(nwg), dim3(256), 0, st, imgs, list, point);
}
size_t png_inflate_smem() { return sizeof(InflateSmem); }

}  // namespace dg
