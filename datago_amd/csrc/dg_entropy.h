// dg_entropy.h — self-synchronising parallel Huffman decoding of a JPEG scan
// (host+device code: the kernels in kernels.hip and the CPU emulator in
// tests/native/ both include it).
//
// Input is the *destuffed* entropy-coded stream of one image (FF00 -> FF,
// RST markers removed, their bit positions listed separately; produced by
// k_destuff_*).  The stream is cut into fixed bit ranges (subsequences)
// [i*S, (i+1)*S).  The decoder of subsequence i decodes every symbol whose
// first bit lies in its range.  Its entry state (bit position of its first
// symbol boundary, block-in-MCU r, zigzag index z) is the exit state of
// subsequence i-1 ("the first symbol boundary at or after i*S").  Started
// from a guessed state, a Huffman decoder falls into step with the true
// decode within a few hundred bits (self-synchronisation; measured in
// DESIGN.md), so a workgroup iterates "re-decode from the predecessor's exit"
// until no exit changes.  An RST marker is a hard sync point: at the first
// symbol boundary at/after it the state resets to (r=0, z=0) and the DC
// predictors reset (T.81 F.2.1.3.1); the marker belongs to the subsequence
// whose range contains its position.
#pragma once
#include "dg_pixel.h"
#include "dg_plane.h"
#include "dg_types.h"

namespace dg {

DG_HD int32_t huff_extend(int32_t v, int32_t s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

DG_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// 64-bit window over a big-endian bit stream stored as bytes (the stream base
// is 4-byte aligned and zero-padded by >= 16 bytes past its end).
//
// Refills are batched per wave.  Behind the window each lane keeps a buffer
// of kBwBuf raw (not yet byte-swapped) words; a shift takes the next one from
// it.  When any lane of a wave has emptied its buffer, every active lane
// reloads its whole buffer at once (bw_refill): one load latency per wave
// every ~kBwBuf words of its fastest lane.  Per-lane refills -- one word
// ahead, issued whenever a lane crossed a word -- stalled the wave on nearly
// every symbol: a wave has one in-order load counter, so the wait for the
// word a lane loaded symbols ago also waited for the loads other lanes had
// issued since.  One symbol consumes at most 31 bits, so with pos - base < 32
// before a symbol at most one 32-bit shift follows it, and a lane with a
// non-empty buffer at the start of a step never runs dry within it.
// Destuffed streams are stored word-interleaved across groups of 64
// subsequences: logical 32-bit word w of subsequence s = w >> lsw (2^lsw
// words per subsequence) sits in row (s / 64) * 2^lsw + (w mod 2^lsw),
// column s mod 64 of a 64-word-wide array.  The 64 lanes of a wave decode
// 64 consecutive subsequences at about the same relative position, so their
// loads hit the same 256-byte rows: coalesced and L2-resident, instead of 64
// lines scattered 2^lsw words apart that the L2 cannot hold for the whole
// batch (PMC: 17x fetch amplification with the plain layout).
DG_HD uint32_t ds_word_index(uint32_t w, uint32_t lsw) {
  const uint32_t s = w >> lsw, j = w & ((1u << lsw) - 1u);
  return ((((s >> 6) << lsw) + j) << 6) + (s & 63u);
}
// physical words needed for a stream of nsub subsequences, plus the margin
// past its end that the zero padding (64 bytes) and a reader's window and
// lookahead reach: >= 1024 bits, and >= 2 subsequences
DG_HD uint64_t ds_words_alloc(uint32_t nsub, uint32_t lsw) {
  const uint32_t margin = ((1024u >> 5) >> lsw) + 2u;
  return ((uint64_t)((nsub + margin + 63u) / 64u) << lsw) * 64;
}

constexpr uint32_t kBwBuf = 6;

struct BitWin {
  const DG_GLOBAL uint32_t *w;  // interleaved stream as little-endian words (byte-swapped on use)
  uint64_t win;       // bits [base, base + 64)
  uint32_t base;      // bit position of win's MSB (multiple of 32)
  uint32_t lsw;       // log2(words per subsequence)
  uint32_t nbuf;      // valid words in buf
  uint32_t buf[kBwBuf];  // raw words base/32 + 2 ..
};

DG_HD uint32_t bw_word(const BitWin &b, uint32_t i) { return b.w[ds_word_index(i, b.lsw)]; }

// buf = the kBwBuf words after the window
DG_HD void bw_fill(BitWin &b) {
  const uint32_t nw = (b.base >> 5) + 2u;
#pragma unroll
  for (uint32_t k = 0; k < kBwBuf; k++) b.buf[k] = bw_word(b, nw + k);
  b.nbuf = kBwBuf;
}

DG_HD void bw_init(BitWin &b, const DG_GLOBAL uint8_t *stream, uint32_t lsw, uint32_t pos) {
  b.w = (const DG_GLOBAL uint32_t *)stream;
  b.lsw = lsw;
  uint32_t i = pos >> 5;
  b.base = i << 5;
  b.win = ((uint64_t)bswap32(bw_word(b, i)) << 32) | bswap32(bw_word(b, i + 1));
  bw_fill(b);
}

// start of a symbol step: no lane may enter it with an empty buffer
DG_HD void bw_refill(BitWin &b) {
#if defined(DG_DEVICE)
  if (__ballot(b.nbuf == 0u)) bw_fill(b);  // wave-uniform: every active lane reloads together
#else
  if (b.nbuf == 0u) bw_fill(b);
#endif
}

// 32 bits starting at pos (requires base <= pos < base + 32).
DG_HD uint32_t bw_peek(const BitWin &b, uint32_t pos) { return (uint32_t)((b.win << (pos - b.base)) >> 32); }

// after a symbol: base <= pos < base + 64 -> base <= pos < base + 32
// (straight-line: the shift is a select, the buffer moves down one word)
DG_HD void bw_shift(BitWin &b, uint32_t pos) {
  const bool adv = pos - b.base >= 32u;
  b.win = adv ? (b.win << 32) | bswap32(b.buf[0]) : b.win;
  b.base += adv ? 32u : 0u;
#pragma unroll
  for (uint32_t k = 0; k + 1 < kBwBuf; k++) b.buf[k] = adv ? b.buf[k + 1] : b.buf[k];
  b.nbuf -= adv ? 1u : 0u;
}

DG_HD void bw_seek(BitWin &b, uint32_t pos) {
  if (pos - b.base >= 32u) bw_init(b, (const DG_GLOBAL uint8_t *)b.w, b.lsw, pos);
}

// Decode one Huffman code from the top bits of `bits`; returns (len << 8) | sym.
template <class T>
DG_HD uint32_t huff_lookup(const T &t, uint32_t bits) {
  uint32_t e = t.lut[bits >> (32 - kLutBits)];
  if (!(e & 0x8000u) && e) return e;
  if (e & 0x8000u) {
    uint32_t e2 = t.sub[e & (kMaxSubTables - 1)][(bits >> (32 - 16)) & ((1u << kSubBits) - 1)];
    return e2 ? e2 : (16u << 8);
  }
  uint32_t pk = bits >> 16;  // fallback for tables with many long prefixes
  for (int32_t l = kLutBits + 1; l <= 16; l++)
    if (pk < t.lim[l]) return ((uint32_t)l << 8) | t.vals[(t.valoff[l] + (int32_t)(pk >> (16 - l))) & 255];
  return 16u << 8;  // invalid code: consume 16 bits (only off-sync / past the data)
}

// First-level lookup, falling back to the sub-tables / lim[] only for codes
// longer than kLutBits (the one branch left in the per-symbol step).
template <class T>
DG_HD uint32_t huff_decode(const T &t, uint32_t bits) {
  const uint32_t e = t.lut[bits >> (32 - kLutBits)];
  if (e != 0u && !(e & 0x8000u)) return e;
  return huff_lookup(t, bits);
}

// Signed value of the `size` magnitude bits that follow a `len`-bit code at
// the top of `bits` (T.81 F.2.2.1 EXTEND); 0 when size == 0.  Branch-free:
// the 64-bit shift by 32 - size yields 0 for size 0.
DG_HD int32_t huff_value(uint32_t bits, uint32_t len, uint32_t size) {
  const uint32_t raw = (uint32_t)((uint64_t)(bits << len) >> (32u - size));
  const uint32_t half = (1u << size) >> 1;
  return raw < half ? (int32_t)raw - (int32_t)((1u << size) - 1u) : (int32_t)raw;
}

// Zigzag position after one symbol decoded at position z: a DC symbol moves
// to 1; an AC symbol to z + run + 1, ZRL (0xF0) to z + 16, EOB to 64.
DG_HD uint32_t huff_next_z(uint32_t z, uint32_t sym) {
  const uint32_t size = sym & 15u, run = sym >> 4;
  const uint32_t zac = (size == 0u && run != 15u) ? 64u : z + run + 1u;
  return z == 0u ? 1u : zac;
}

// ---- multi-symbol AC steps for the state-only decodes (lead-in, sync)
//
// The state-only decodes need no AC values, only where the symbols end.  A
// per-AC-table lookup on the next kMultiBits stream bits gives how many of
// them the AC symbols (code + magnitude bits) that fit entirely inside take,
// their zigzag advance, and whether the last one was EOB:
//   entry = bits (0 = none fits) | advance << 4 | eob << 11
// A step takes the entry instead of one symbol when the whole run stays in
// the block and ends at or before the next event, so it passes exactly the
// symbol boundaries single steps would: the same states, fewer steps.
#ifndef DG_MULTI_BITS
#define DG_MULTI_BITS 11  // 10 / 11 / 12 measured: huff_sync 1.77 / 1.63 / 1.75 ms (experiment builds: DG_HIPCC_FLAGS=-DDG_MULTI_BITS=n, n <= 15)
#endif
constexpr uint32_t kMultiBits = DG_MULTI_BITS;
constexpr uint32_t kMultiLuts = 3;  // distinct AC tables per image

template <class TAB>
DG_HD uint32_t multi_entry(const TAB &t, uint32_t pfx) {
  const uint32_t bits = pfx << (32u - kMultiBits);
  uint32_t o = 0, adv = 0, eob = 0;
  while (o < kMultiBits) {
    const uint32_t e = huff_lookup(t, bits << o);
    const uint32_t len = e >> 8, sym = e & 0xFFu, size = sym & 15u, run = sym >> 4;
    if (len == 0u || len >= 16u || o + len + size > kMultiBits) break;  // invalid, or not inside the window
    if (size == 0u && run != 15u) {  // EOB
      o += len;
      eob = 1;
      break;
    }
    const uint32_t nadv = adv + (size == 0u ? 16u : run + 1u);
    if (nadv > 64u) break;
    adv = nadv;
    o += len + size;
    if (adv == 64u) break;  // the block ends with this coefficient
  }
  return o | (adv << 4) | (eob << 11);
}

// z after a multi entry m taken at z, or 0xFFFFFFFF if it cannot be taken
// there (no symbol fits, or the run would leave the block)
DG_HD uint32_t multi_next_z(uint32_t m, uint32_t z) {
  const uint32_t c = m & 15u, adv = (m >> 4) & 127u, eob = (m >> 11) & 1u;
  const bool ok = c != 0u && z != 0u && (eob ? z + adv < 64u : z + adv <= 64u);
  return ok ? (eob ? 64u : z + adv) : 0xFFFFFFFFu;
}

// Accumulators of one subsequence decode.
struct RangeAcc {
  uint32_t out;
  uint32_t m, n;
  int32_t dc[3];
};

// Write-side context: coefficient block buffer of this thread (64 int16,
// zigzag order), global coefficient base, prefix values.
// k_huff_write's block buffers are 128 bytes apart with their 16-byte parts
// XOR-swizzled by the owner lane: coefficient zz sits at blk[zz ^ sw], sw =
// ((lane >> 1) & 7) << 3, so the 16-byte accesses of 16 consecutive lanes
// cover all 64 banks (the unswizzled 128-byte stride put them on two groups
// of four).  72-int16 buffers did the same with 12% more LDS; at 64 the
// kernel fits three workgroups per CU instead of two.
struct WriteCtx {
  int16_t *blk;
  uint32_t sw = 0;  // swizzle of this thread's buffer (int16 units; 0 on the host)
  DG_GLOBAL int16_t *coef;
  uint32_t seg, nin;
  int32_t pred[3];
  uint32_t blocks_per_seg, total_blocks;
  int32_t cur;   // global index of the block being filled (-1 = none / dropped)
  uint32_t zs;   // first zigzag index this thread owns in the current block
#if defined(DG_DEVICE)
  // sparse blocks (ImageDesc::ccnt): per block, the mask of the 16-byte
  // parts stored (the nonzero ones); nullptr = dense (all 8 parts)
  DG_GLOBAL uint8_t *cnt = nullptr;
  // wave-cooperative flush (k_huff_write): this wave's lane-0 block, block
  // stride (int16), and a 128-dword LDS table of the wave
  int16_t *wave_blk;
  uint32_t stride;
  uint32_t *tab;
  // fused IDCT (ImageDesc::idct_fused): completed blocks become plane pixels
  const ImageDesc *im;      // nullptr: blocks are written as coefficients
  const int32_t *qt;        // LDS: the image's quantisation tables, [component][natural index]
  const uint8_t *n2z;       // LDS: natural index -> zigzag index
  BatchFlags *flags;        // idct_late / idct_list: blocks left to k_idct_list
  uint32_t img;             // descriptor index
#endif
};

DG_HD int32_t wc_index(const WriteCtx &w, uint32_t in_seg) {
  if (w.blocks_per_seg && in_seg >= w.blocks_per_seg) return -1;
  uint64_t g = (uint64_t)(w.blocks_per_seg ? w.seg : 0) * w.blocks_per_seg + in_seg;
  return g < w.total_blocks ? (int32_t)g : -1;
}

DG_HD void wc_begin(WriteCtx &w, int32_t idx, uint32_t zs) {
  w.cur = idx;
  w.zs = zs;
#if defined(DG_DEVICE)
  u32x4 *p = (u32x4 *)w.blk;
  const u32x4 zero = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = zero;
#else
  for (int i = 0; i < 64; i++) w.blk[i] = 0;
#endif
}

DG_HD void wc_flush(WriteCtx &w, uint32_t ze) {
  if (w.cur < 0) return;
  DG_GLOBAL int16_t *dst = w.coef + (size_t)w.cur * 64;
  if (w.zs == 0 && ze == 64) {
#if defined(DG_DEVICE)
    const u32x4 *s4 = (const u32x4 *)w.blk;
    DG_GLOBAL u32x4 *d4 = (DG_GLOBAL u32x4 *)dst;
#pragma unroll
    for (int i = 0; i < 8; i++) d4[i] = s4[i ^ (w.sw >> 3)];
#else
    for (int i = 0; i < 64; i++) dst[i] = w.blk[i ^ w.sw];
#endif
  } else {
    for (uint32_t i = w.zs; i < ze; i++) dst[i] = w.blk[i ^ w.sw];
  }
#if defined(DG_DEVICE)
  // a block shared by two ranges (or cut at the range end) is stored dense:
  // each owner writes its zigzag span and both announce all 8 parts
  if (w.cnt) w.cnt[w.cur] = 0xFFu;
#endif
  w.cur = -1;
}

#if defined(DG_DEVICE)
// Fused IDCT: a block whose coefficients reach the coefficient buffer (not
// IDCT-ed in the flush) is listed for k_idct_list.
__device__ __forceinline__ void wc_list_late(WriteCtx &w, int32_t idx) {
  if (!w.im || idx < 0) return;
  const uint32_t e = atomicAdd(&w.flags->idct_late, 1u);
  if (e < w.flags->idct_cap) {
    uint32_t *l = (uint32_t *)(uintptr_t)w.flags->idct_list;
    l[2 * e] = w.img;
    l[2 * e + 1] = (uint32_t)idx;
  }
}

// Full blocks completed by lanes of a wave are written out together: a lane
// whose block ends only marks it pending, and at the top of the next symbol
// step the wave's active lanes copy every pending block with one 16-byte
// chunk each (8 lanes per block, 128 contiguous bytes) and zero it in LDS for
// its owner's next block.  A per-lane flush costs every lane 8 LDS loads, 8
// global stores and 8 LDS stores whenever any lane of the wave ends a block,
// which with ~8 symbols per block is nearly every step.  Blocks are zero
// whenever a lane has none open, so a block start only sets its index.
__device__ __forceinline__ void wc_coop_flush(WriteCtx &w, bool pending) {
  const uint64_t pm = __ballot(pending);
  if (!pm) return;
  const uint64_t am = __ballot(1);
  if (pending) {
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
    w.tab[rank] = __lane_id();  // bits 8..15: the nonzero parts (sparse flushes OR them in)
    w.tab[64 + rank] = (uint32_t)w.cur;
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t wr = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
  const uint32_t na = (uint32_t)__popcll(am), nb = (uint32_t)__popcll(pm), nc = 8u * nb;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  if (w.im && na >= 8) {
    // Fused IDCT: groups of 8 active lanes take one pending block each per
    // round; lane `part` runs column `part` (dequantised from the zigzag
    // coefficients) of pass 1, the 8 workspace columns go back into the
    // block's own LDS buffer in natural order, then lane `part` runs row
    // `part` of pass 2 and stores 8 plane pixels.  All 8 lanes of a block
    // are in the same round, so every pass-1 read precedes the writes
    // (one wave: LDS operations in program order).
    const ImageDesc &im = *w.im;
    const bool zune = im.sem != 0;
    const uint32_t groups = na >> 3, g = wr >> 3, part = wr & 7u;
    for (uint32_t k0 = 0; k0 < nb; k0 += groups) {
      const uint32_t k = k0 + g;
      const bool act = g < groups && k < nb;
      const int32_t idx = act ? (int32_t)w.tab[64 + k] : -1;
      const uint32_t own = act ? w.tab[k] & 255u : 0u;
      int16_t *b = w.wave_blk + own * w.stride;
      const uint32_t osw = w.stride == 64u ? ((own >> 1) & 7u) << 3 : 0u;  // the owner's swizzle
      const bool live = act && idx >= 0;
      uint32_t c = 0, by = 0, bx = 0;
      if (live) block_pos(im, (uint32_t)idx, c, by, bx);
      int32_t ws[8];
      if (live) {
        int32_t v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = (int32_t)b[w.n2z[r * 8 + part] ^ osw] * w.qt[c * 64 + r * 8 + part];
        idct_col(zune, v, ws);
      }
      __builtin_amdgcn_wave_barrier();
      if (live) {
#pragma unroll
        for (int r = 0; r < 8; r++) b[r * 8 + part] = (int16_t)ws[r];
      }
      __builtin_amdgcn_wave_barrier();
      if (act) {
        u32x4 *row4 = (u32x4 *)b + part;
        if (live) {
          const u32x4 rv = *row4;
          int16_t h[8];
          __builtin_memcpy(h, &rv, 16);
          int32_t row[8];
          uint32_t px[8];
#pragma unroll
          for (int i = 0; i < 8; i++) row[i] = h[i];
          idct_row(zune, row, px);
          store_plane_row8(im, c, by * 8 + part, bx, px);  // plain plane or chroma records (dg_plane.h)
        }
        *row4 = zero;
      }
      __builtin_amdgcn_wave_barrier();
    }
    return;
  }
  for (uint32_t c = wr; c < nc; c += na) {
    const uint32_t k = c >> 3, part = c & 7u;
    const int32_t idx = (int32_t)w.tab[64 + k];
    const uint32_t own = w.tab[k] & 255u;
    u32x4 *src = (u32x4 *)(w.wave_blk + own * w.stride) + (w.stride == 64u ? part ^ ((own >> 1) & 7u) : part);
    const u32x4 v = *src;
    // sparse blocks: an all-zero part is not stored; the parts that are go
    // into the block's mask (k_idct_t loads those, the rest read as zero)
    const bool nz = (v.x | v.y | v.z | v.w) != 0u;
    if (idx >= 0 && (nz || !w.cnt)) *(DG_GLOBAL u32x4 *)(w.coef + (size_t)idx * 64 + part * 8) = v;
    if (w.cnt && nz) atomicOr(&w.tab[k], 256u << part);
    *src = zero;
    if (part == 0) wc_list_late(w, idx);  // fused IDCT with < 8 active lanes: k_idct_list takes it
  }
  __builtin_amdgcn_wave_barrier();
  if (w.cnt && wr < nb) {  // one lane per flushed block: its mask
    const int32_t idx = (int32_t)w.tab[64 + wr];
    if (idx >= 0) w.cnt[idx] = (uint8_t)(w.tab[wr] >> 8);
  }
  __builtin_amdgcn_wave_barrier();
}

// rare paths (partial blocks at range ends and restart markers): flush, then
// restore the all-zero block
__device__ __forceinline__ void wc_flush_zero(WriteCtx &w, uint32_t ze) {
  wc_flush(w, ze);
  u32x4 *p = (u32x4 *)w.blk;
  const u32x4 zero = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = zero;
}
#endif

// Block flush / start inside decode_range: wave-cooperative on the device
// when the context provides the table (COOP), per lane otherwise.
template <bool COOP>
DG_HD void wc_end_block(WriteCtx &w, bool &pending) {
#if defined(DG_DEVICE)
  if (COOP) {
    if (w.zs == 0) {
      pending = true;
    } else {  // carried in from the previous range: its first coefficients are in the buffer already
      const int32_t idx = w.cur;
      wc_flush_zero(w, 64);
      wc_list_late(w, idx);
    }
    return;
  }
#endif
  (void)pending;
  wc_flush(w, 64);
}
template <bool COOP>
DG_HD void wc_partial(WriteCtx &w, uint32_t ze) {
#if defined(DG_DEVICE)
  if (COOP) {
    wc_flush_zero(w, ze);
    return;
  }
#endif
  wc_flush(w, ze);
}

// Decode-once staging (option "entropy_once").  The sync decode records
// every coefficient it produces, so k_huff_scatter writes the blocks without
// decoding the range a second time.  Entries are 32-bit:
//   coefficient  bit 31 = 0 | zz:6 @25 | j:13 @12 | value:12 (signed) @0
//   RST marker   bit 31 = 1 | owned @30 | z:6 @24 | j:13 @11
// j = blocks started in the range so far (0: the block carried in from the
// previous range), z = zigzag position when the marker was reached.  DC
// differences of 0 are not recorded.  Groups of four entries are stored
// interleaved over 64 consecutive ranges (group g of range s at
// ((s / 64) * cap + g) * 64 + s % 64, 16 bytes each) so that a wave's loads
// and stores of its g-th groups coalesce.
struct StageCtx {
  DG_GLOBAL uint32_t *base;  // this range's group 0
  uint32_t on;               // this thread stages (decode_range checks it; the context itself is always passed
                             // by the staging kernels, so it stays in registers)
  uint32_t n, started;       // entries, blocks started
  uint32_t g0, g1, g2, g3;   // pending group
};
DG_HD uint32_t stage_coef(uint32_t zz, uint32_t j, int32_t v) {
  return (zz << 25) | ((j & 0x1FFFu) << 12) | ((uint32_t)v & 0xFFFu);
}
DG_HD uint32_t stage_marker(uint32_t owned, uint32_t z, uint32_t j) {
  return 0x80000000u | (owned << 30) | ((z & 63u) << 24) | ((j & 0x1FFFu) << 11);
}
DG_HD DG_GLOBAL uint32_t *stage_range(uint64_t stage, uint32_t cap, uint32_t s) {
  return (DG_GLOBAL uint32_t *)(uintptr_t)stage + ((((size_t)(s >> 6) * cap) << 6) + (s & 63u)) * 4;
}
DG_HD void stage_push(StageCtx &c, uint32_t e) {
  const uint32_t k = c.n & 3u;
  c.g0 = k == 0 ? e : c.g0;
  c.g1 = k == 1 ? e : c.g1;
  c.g2 = k == 2 ? e : c.g2;
  c.g3 = k == 3 ? e : c.g3;
  c.n++;
  if (k == 3) {
    DG_GLOBAL uint32_t *p = c.base + (size_t)((c.n >> 2) - 1) * 256;  // 64 ranges x 4 dwords per group row
#if defined(DG_DEVICE)
    *(DG_GLOBAL u32x4 *)p = u32x4{c.g0, c.g1, c.g2, c.g3};
#else
    p[0] = c.g0, p[1] = c.g1, p[2] = c.g2, p[3] = c.g3;
#endif
  }
}
DG_HD void stage_finish(StageCtx &c) {
  if (c.n & 3u) {
    DG_GLOBAL uint32_t *p = c.base + (size_t)(c.n >> 2) * 256;
#if defined(DG_DEVICE)
    *(DG_GLOBAL u32x4 *)p = u32x4{c.g0, c.g1, c.g2, c.g3};
#else
    p[0] = c.g0, p[1] = c.g1, p[2] = c.g2, p[3] = c.g3;
#endif
  }
}

// Checkpoints for early merging.  A decode records, at the first symbol
// boundary at/after every kCkptBits-th bit of its range, the state there and
// the accumulator *tail* from that point to the end of the range.  A later
// re-decode of the same range from a different entry state compares states at
// each checkpoint: once they agree the two paths coincide to the end, so it
// stops and completes its totals with the stored tail.  This cuts a re-decode
// from a full range to about the self-synchronisation distance.
constexpr uint32_t kCkptBits = 256;
// enough for sub_bits <= 4096, and for the half-way checkpoint of an
// 8192-bit range (index 15), where k_huff_write splits a range (write_split).
// (32, for split 16384-bit ranges: sub_auto 16384 measured no faster,
// profiles/r04/sub16k)
constexpr uint32_t kMaxCkpt = 16;
struct Ckpt {
  uint32_t st;   // packed state (rel past the checkpoint position, r, z)
  uint32_t m, n; // tail (segmented: m > 0 means the tail contains a reset)
  int32_t dc[3];
};

DG_HD uint32_t num_ckpt(uint32_t sub_bits) {
  uint32_t k = (sub_bits - 1) / kCkptBits;
  return k > kMaxCkpt ? kMaxCkpt : k;
}

// Position of the first RST marker >= pos in the image's sorted marker list.
DG_HD uint32_t first_marker(const DG_GLOBAL uint32_t *mk, uint32_t nmk, uint32_t pos, uint32_t &idx) {
  uint32_t lo = 0, hi = nmk;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (mk[mid] < pos) lo = mid + 1;
    else hi = mid;
  }
  idx = lo;
  return lo < nmk ? mk[lo] : kInf;
}

// Entry-state guess for subsequence s: decode (state only) from `lead` bits
// before its start — from a guessed MCU start there, or exactly from the
// scan start / a restart marker when one is closer — up to the first symbol
// boundary at or after the start.  JPEG decodes self-synchronise within a few
// hundred to a few thousand bits (tools/sync_stats.cpp; slowest for 4:2:0,
// whose 6-block MCU phase must also lock), so with a long enough lead the
// guess is the true state and k_huff_sync's verification loop has nothing to
// re-decode.
template <class TAB>
DG_HD uint32_t lead_in(const ImageDesc &im, const TAB *tabs, const DG_GLOBAL uint8_t *stream,
                       const DG_GLOBAL uint32_t *mk, uint32_t s, uint32_t lead,
                       const uint16_t *mt = nullptr, uint32_t acm = 0xFFu, bool pair = false) {
  const uint32_t a0 = s * im.sub_bits;
  if (s == 0 || lead == 0 || a0 >= im.ds_bits) return pack_state(0, 0, 0);
  uint32_t pos = a0 > lead ? a0 - lead : 0u;
  uint32_t r = 0, z = 0, midx;
  uint32_t mpos = im.nmk ? first_marker(mk, im.nmk, pos, midx) : kInf;
  const uint32_t bpm = im.bpm, slotmap = im.slotmap, cbits = im.comp_bits;
  uint32_t comp = cbits & 3u;
  // the current block's DC/AC tables, resolved when the block changes
  const TAB *tdc = &tabs[(slotmap >> ((comp << 1) << 2)) & 15u];
  const TAB *tac = &tabs[(slotmap >> (((comp << 1) | 1u) << 2)) & 15u];
  // multi-symbol table of the block's AC table (acm: 2 bits per component, 3 = none)
  uint32_t mi = mt ? (acm >> (2u * comp)) & 3u : 3u;
  BitWin b;
  bw_init(b, stream, im.ds_lsw, pos);
  for (;;) {
    if (pos >= mpos) {  // restart marker before the start: exact state from here
      pos = mpos;
      r = 0;
      z = 0;
      comp = cbits & 3u;
      tdc = &tabs[(slotmap >> ((comp << 1) << 2)) & 15u];
      tac = &tabs[(slotmap >> (((comp << 1) | 1u) << 2)) & 15u];
      mi = mt ? (acm >> (2u * comp)) & 3u : 3u;
      midx++;
      mpos = midx < im.nmk ? mk[midx] : kInf;
      bw_seek(b, pos);
    }
    if (pos >= a0) break;
    bw_refill(b);
    // state-only step, straight-line apart from the long-code lookup and the
    // refill (with 64 lanes in different places of their blocks, a branch per
    // case would run every case every step): one symbol, or a multi-symbol
    // AC run that ends at or before the next event (start or marker)
    const uint32_t bits = bw_peek(b, pos);
    const uint32_t e = huff_decode(*(z == 0u ? tdc : tac), bits);
    const uint32_t m = (mi != 3u && z != 0u) ? (uint32_t)mt[(mi << kMultiBits) | (bits >> (32u - kMultiBits))] : 0u;
    const uint32_t sym = e & 0xFFu;
    const uint32_t zm = multi_next_z(m, z);
    const uint32_t lim = a0 < mpos ? a0 : mpos;
    const bool take_m = zm != 0xFFFFFFFFu && pos + (m & 15u) <= lim;
    pos += take_m ? (m & 15u) : (e >> 8) + (sym & 15u);
    uint32_t zn = take_m ? zm : huff_next_z(z, sym);
    if (pair && !take_m) {  // a second AC symbol from the same peek (see decode_range)
      const uint32_t c1 = (e >> 8) + (sym & 15u);
      const bool eob1 = z != 0u && (sym & 15u) == 0u && (sym >> 4) != 15u;
      const uint32_t bits2 = c1 < 32u ? bits << c1 : 0u;
      const uint32_t e2 = huff_decode(*tac, bits2);
      const uint32_t sym2 = e2 & 0xFFu, c2 = (e2 >> 8) + (sym2 & 15u);
      if (!eob1 && zn < 64u && pos < lim && c1 + c2 <= 32u) {
        pos += c2;
        zn = huff_next_z(zn, sym2);
      }
    }
    bw_shift(b, pos);
    const bool bend = zn >= 64u;
    z = bend ? 0u : zn;
    r = bend ? (r + 1u == bpm ? 0u : r + 1u) : r;
    comp = (cbits >> (2u * r)) & 3u;
    tdc = &tabs[(slotmap >> ((comp << 1) << 2)) & 15u];
    tac = &tabs[(slotmap >> (((comp << 1) | 1u) << 2)) & 15u];
    mi = mt ? (acm >> (2u * comp)) & 3u : 3u;
  }
  const uint32_t rel = pos - a0;
  return pack_state(rel > 255 ? 255 : rel, r, z);
}

// Decode the symbols of subsequence s of image im from entry state `in`.
//   stream: destuffed bytes (4-byte aligned, zero padded); mk: marker bit positions
//   tabs: Huffman tables indexed by slot (im.dc_slot / im.ac_slot)
//   ck: this subsequence's checkpoint records (nullptr: none); merge: the
//   records hold a previous decode of this range whose exit state was old_out.
template <bool WRITE, class TAB, bool COOP = false>
DG_HD void decode_range(const ImageDesc &im, const TAB *tabs, const DG_GLOBAL uint8_t *stream,
                        const DG_GLOBAL uint32_t *mk,
                        uint32_t s, uint32_t in, RangeAcc &acc, WriteCtx *w, DG_GLOBAL Ckpt *ck = nullptr,
                        bool merge = false, uint32_t old_out = 0, StageCtx *stg = nullptr,
                        const uint16_t *mt = nullptr, uint32_t acm = 0xFFu, uint32_t pair = 0,
                        uint32_t a0o = kInf, uint32_t a1o = kInf) {
  // [a0o, a1o): a part of the range (k_huff_write's split halves); `in` is
  // then the state at the first symbol boundary at/after a0o
  const uint32_t S = im.sub_bits, total = im.ds_bits;
  const uint32_t r0 = s * S;
  const uint32_t a0 = a0o != kInf ? a0o : r0;
  const uint32_t a1 = a1o != kInf ? a1o : ((r0 + S < total) ? r0 + S : total);
  uint32_t r = st_r(in), z = st_z(in);
  uint32_t pos = a0 + st_rel(in);
  acc.m = 0;
  acc.n = 0;
  acc.dc[0] = acc.dc[1] = acc.dc[2] = 0;
  const bool stage = stg && stg->on;
  if (stage) {
    stg->n = 0;
    stg->started = 0;
  }
  if (a0 >= total) {  // empty trailing subsequence (nsub is sized from the raw length):
    acc.out = pack_state(0, 0, 0);  // constant exit, so state changes do not ripple through it
    return;
  }
  uint32_t midx;
  uint32_t mpos = im.nmk ? first_marker(mk, im.nmk, a0, midx) : kInf;
  const uint32_t bpm = im.bpm;
  const uint32_t slotmap = im.slotmap;  // 4 bits per (component, dc/ac)
  BitWin b;
  bw_init(b, stream, im.ds_lsw, pos < a1 ? pos : a0);
  const uint32_t cbits = im.comp_bits;
  uint32_t comp = (cbits >> (2 * r)) & 3u;
  const uint32_t nck = ck ? num_ckpt(S) : 0;
  uint32_t k = 0, cpos = a0 + kCkptBits;
  bool merged = false;
  bool pending = false;  // COOP: a completed block awaits the wave's flush
  if (WRITE) {
    w->cur = -1;
    if (z > 0) wc_begin(*w, w->nin > 0 ? wc_index(*w, w->nin - 1) : -1, z);
  }
  // Per symbol only one compare against the next "event" (restart marker,
  // checkpoint, end of range); the Huffman tables of the current block are
  // resolved when the block changes, not per symbol.
  auto next_event = [&]() -> uint32_t {
    uint32_t e = a1 < mpos ? a1 : mpos;
    return (k < nck && cpos < e) ? cpos : e;
  };
  // multi-symbol AC steps (state-only passes: no AC values written or staged)
  const bool multi = !WRITE && !stage && mt != nullptr;
  uint32_t mi = 3u;
  auto block_tables = [&](const TAB *&tdc, const TAB *&tac) {
    tdc = &tabs[(slotmap >> ((comp << 1) << 2)) & 15u];
    tac = &tabs[(slotmap >> (((comp << 1) | 1u) << 2)) & 15u];
    mi = multi ? (acm >> (2u * comp)) & 3u : 3u;
  };
  const TAB *tdc, *tac;
  block_tables(tdc, tac);
  uint32_t ev = next_event();
  for (;;) {
#if defined(DG_DEVICE)
    if (WRITE && COOP) {
      wc_coop_flush(*w, pending);
      pending = false;
    }
#endif
    if (pos >= ev) {
      if (pos >= mpos) {  // restart marker: hard resync
        bool owned = mpos < a1;
        if (WRITE && z > 0) wc_partial<COOP>(*w, z);
        if (stage) stage_push(*stg, stage_marker(owned ? 1u : 0u, z, stg->started));
        pos = mpos;
        r = 0;
        z = 0;
        comp = cbits & 3u;
        block_tables(tdc, tac);
        if (owned) {
          acc.m++;
          acc.n = 0;
          acc.dc[0] = acc.dc[1] = acc.dc[2] = 0;
          if (WRITE) {
            w->seg++;
            w->nin = 0;
            w->pred[0] = w->pred[1] = w->pred[2] = 0;
          }
        }
        midx++;
        mpos = midx < im.nmk ? mk[midx] : kInf;
        bw_seek(b, pos);
      }
      if (k < nck && cpos < a1 && pos >= cpos) {  // first boundary at/after checkpoint k
        uint32_t rel = pos - cpos;
        uint32_t st = pack_state(rel > 255 ? 255 : rel, r, z);
        DG_GLOBAL Ckpt &c = ck[k];
        if (merge && c.st == st) {  // rejoined the previous decode: acc (+) tail_k
          if (c.m) {
            acc.m += c.m;
            acc.n = c.n;
            acc.dc[0] = c.dc[0];
            acc.dc[1] = c.dc[1];
            acc.dc[2] = c.dc[2];
          } else {
            acc.n += c.n;
            acc.dc[0] += c.dc[0];
            acc.dc[1] += c.dc[1];
            acc.dc[2] += c.dc[2];
          }
          acc.out = old_out;
          merged = true;
          break;
        }
        c.st = st;  // record the prefix for now; turned into a tail at the end
        c.m = acc.m;
        c.n = acc.n;
        c.dc[0] = acc.dc[0];
        c.dc[1] = acc.dc[1];
        c.dc[2] = acc.dc[2];
        k++;
        cpos += kCkptBits;
      }
      if (pos >= a1) break;
      ev = next_event();
    }
    // One symbol.  Straight-line apart from the long-code lookup, the refill
    // and the write pass's rare partial flush: the 64 lanes of a wave sit at
    // different places of their blocks, so a branch per case (DC / AC / block
    // end) would run every case in every step anyway, plus the exec-mask
    // bookkeeping.
    bw_refill(b);
    const uint32_t bits = bw_peek(b, pos);
    const bool isdc = (z == 0);
    const uint32_t e = huff_decode(*(isdc ? tdc : tac), bits);
    const uint32_t len = e >> 8, sym = e & 0xFFu;
    const uint32_t size = sym & 15u;
    const uint32_t run = isdc ? 0u : (sym >> 4);
    const int32_t v = huff_value(bits, len, size);
    uint32_t zm = 0xFFFFFFFFu, mc = 0;
    if (!WRITE) {  // an AC run ending at or before the next event: same boundaries as single steps
      const uint32_t m = (mi != 3u && !isdc) ? (uint32_t)mt[(mi << kMultiBits) | (bits >> (32u - kMultiBits))] : 0u;
      mc = m & 15u;
      zm = pos + mc <= ev ? multi_next_z(m, z) : 0xFFFFFFFFu;
    }
    const bool take_m = zm != 0xFFFFFFFFu;
    pos += take_m ? mc : len + size;
    const int32_t vdc = isdc ? v : 0;
    acc.n += isdc ? 1u : 0u;
    add3(acc.dc, comp, vdc);
    if (stage) {
      if (isdc) {
        stg->started++;
        if (v) stage_push(*stg, stage_coef(0, stg->started, v));
      } else if (size && z + run < 64) {
        stage_push(*stg, stage_coef(z + run, stg->started, v));
      }
    }
    if (WRITE) {
      add3(w->pred, comp, vdc);
      if (isdc) {
        if (COOP) {
          w->cur = wc_index(*w, w->nin);
          w->zs = 0;
        } else {
          wc_begin(*w, wc_index(*w, w->nin), 0);
        }
        w->nin++;
      }
      const uint32_t zz = z + run;
      if (isdc || (size && zz < 64u)) w->blk[zz ^ w->sw] = (int16_t)(isdc ? sel3(w->pred, comp) : v);
    }
    uint32_t zn = take_m ? zm : huff_next_z(z, sym);
    if (pair && !stage && (WRITE || !take_m)) {
      // Further AC symbols of the same block out of the same 32-bit peek
      // (up to `pair` more), each when the block is still open, it starts
      // before the next event and it fits in the peek: exactly the symbols
      // the next single steps would decode.  (The state-only sync decode
      // takes them only after a single symbol.)
      uint32_t used = len + size;
      bool open = isdc || !(size == 0u && run != 15u);  // not EOB
#pragma unroll
      for (uint32_t x = 0; x < 3u; x++) {
        if (x >= pair) break;
        const uint32_t bx = used < 32u ? bits << used : 0u;
        const uint32_t ex = huff_decode(*tac, bx);
        const uint32_t lx = ex >> 8, sx = ex & 0xFFu, zx = sx & 15u;
        const bool tk = open && zn < 64u && pos < ev && used + lx + zx <= 32u;
        if (tk) {
          if (WRITE) {
            const uint32_t zz2 = zn + (sx >> 4);
            if (zx && zz2 < 64u) w->blk[zz2 ^ w->sw] = (int16_t)huff_value(bx, lx, zx);
          }
          pos += lx + zx;
          used += lx + zx;
          zn = huff_next_z(zn, sx);
        }
        open = tk && !(zx == 0u && (sx >> 4) != 15u);
      }
    }
    bw_shift(b, pos);  // one shift: both symbols came out of one peek (< 32 bits past it)
    const bool bend = zn >= 64u;
    if (WRITE && bend) wc_end_block<COOP>(*w, pending);
    z = bend ? 0u : zn;
    r = bend ? (r + 1u == bpm ? 0u : r + 1u) : r;
    comp = (cbits >> (2u * r)) & 3u;
    block_tables(tdc, tac);
  }
  if (WRITE && z > 0) wc_partial<COOP>(*w, z);
  if (stage) stage_finish(*stg);
  if (!merged) {
    uint32_t rel = pos - a1;
    acc.out = pack_state(rel > 255 ? 255 : rel, r, z);
  }
  for (uint32_t j = 0; j < k; j++) {  // prefixes written this time -> tails
    DG_GLOBAL Ckpt &c = ck[j];
    if (acc.m > c.m) {
      c.m = acc.m - c.m;
      c.n = acc.n;
      c.dc[0] = acc.dc[0];
      c.dc[1] = acc.dc[1];
      c.dc[2] = acc.dc[2];
    } else {
      c.m = 0;
      c.n = acc.n - c.n;
      c.dc[0] = acc.dc[0] - c.dc[0];
      c.dc[1] = acc.dc[1] - c.dc[1];
      c.dc[2] = acc.dc[2] - c.dc[2];
    }
  }
}

// ---- two state-only chains per lane (k_huff_sync2)
//
// k_huff_sync's per-lane work -- the lead-in of subsequence s (lead_in) and
// then its range (decode_range<false>: counts, DC sums, checkpoints, exit
// state) -- is one serial chain of dependent table lookups.  With few waves
// per SIMD (a configs[1] batch has ~3 per SIMD, dg_decode_one's small
// batches one) nothing hides a lookup's LDS latency.
// SyncChain is that chain as a resumable state machine, so that a lane can
// advance two independent chains (subsequences s and s + 128) in lockstep
// and both chains' lookups are in flight together.  The step is
// decode_range's state-only step with multi-symbol AC runs; the rare events
// (restart markers, checkpoints, the end of the lead-in and of the range)
// run in a per-chain branch, in decode_range's order.  A finished chain
// keeps stepping with its position frozen -- only the position and the
// counts are guarded per step -- and its results were fixed when it finished.
// tests/native/emu.cpp checks every pair against lead_in + decode_range.
template <class TAB>
struct SyncChain {
  BitWin b;
  uint32_t pos, r, z, comp, mi, ev;
  uint32_t phase;  // 0 lead-in, 1 range, 2 done
  uint32_t a0, a1, mpos, midx, k, cpos, nck;
  uint32_t in;     // entry state of the range (the lead-in's exit)
  const TAB *tdc, *tac;
  RangeAcc acc;    // the range's accumulators (final once phase == 2)
  DG_GLOBAL Ckpt *ck;
};

template <class TAB>
DG_HD void schain_tables(SyncChain<TAB> &c, const ImageDesc &im, const TAB *tabs, const uint16_t *mt, uint32_t acm) {
  c.tdc = &tabs[(im.slotmap >> ((c.comp << 1) << 2)) & 15u];
  c.tac = &tabs[(im.slotmap >> (((c.comp << 1) | 1u) << 2)) & 15u];
  c.mi = mt ? (acm >> (2u * c.comp)) & 3u : 3u;
}

// range phase from entry state c.in (decode_range's prologue); `fresh`: the
// bit window is not positioned yet (no lead-in ran)
template <class TAB>
DG_HD void schain_range(SyncChain<TAB> &c, const ImageDesc &im, const TAB *tabs, const DG_GLOBAL uint8_t *stream,
                        const DG_GLOBAL uint32_t *mk, const uint16_t *mt, uint32_t acm, bool fresh) {
  c.phase = 1;
  c.acc.m = 0;
  c.acc.n = 0;
  c.acc.dc[0] = c.acc.dc[1] = c.acc.dc[2] = 0;
  c.r = st_r(c.in);
  c.z = st_z(c.in);
  if (c.a0 >= im.ds_bits) {  // empty trailing subsequence: constant exit
    c.acc.out = pack_state(0, 0, 0);
    c.phase = 2;
    c.ev = kInf;
    if (fresh) {  // a valid window for the frozen steps
      c.pos = 0;
      bw_init(c.b, stream, im.ds_lsw, 0);
    }
    return;
  }
  c.pos = c.a0 + st_rel(c.in);
  c.mpos = im.nmk ? first_marker(mk, im.nmk, c.a0, c.midx) : kInf;
  if (fresh) bw_init(c.b, stream, im.ds_lsw, c.pos < c.a1 ? c.pos : c.a0);
  c.comp = (im.comp_bits >> (2 * c.r)) & 3u;
  schain_tables(c, im, tabs, mt, acm);
  c.k = 0;
  c.cpos = c.a0 + kCkptBits;
  const uint32_t e = c.a1 < c.mpos ? c.a1 : c.mpos;
  c.ev = (c.k < c.nck && c.cpos < e) ? c.cpos : e;
}

template <class TAB>
DG_HD void schain_begin(SyncChain<TAB> &c, const ImageDesc &im, const TAB *tabs, const DG_GLOBAL uint8_t *stream,
                        const DG_GLOBAL uint32_t *mk, uint32_t s, uint32_t lead, bool active, DG_GLOBAL Ckpt *ck,
                        const uint16_t *mt, uint32_t acm) {
  const uint32_t S = im.sub_bits, total = im.ds_bits;
  c.ck = ck;
  c.nck = ck ? num_ckpt(S) : 0u;
  c.a0 = s * S;
  c.a1 = c.a0 + S < total ? c.a0 + S : total;
  c.k = 0;
  c.cpos = 0;
  c.midx = 0;
  c.mpos = kInf;
  c.in = pack_state(0, 0, 0);
  c.acc.out = pack_state(0, 0, 0);
  c.acc.m = c.acc.n = 0;
  c.acc.dc[0] = c.acc.dc[1] = c.acc.dc[2] = 0;
  c.r = c.z = 0;
  c.comp = im.comp_bits & 3u;
  if (!active) {  // no subsequence: a finished chain on a valid window
    c.phase = 2;
    c.ev = kInf;
    c.pos = 0;
    bw_init(c.b, stream, im.ds_lsw, 0);
    schain_tables(c, im, tabs, mt, acm);
    return;
  }
  if (s == 0 || lead == 0 || c.a0 >= total) {  // lead_in's exact / constant entry
    schain_range(c, im, tabs, stream, mk, mt, acm, true);
    return;
  }
  c.phase = 0;
  c.pos = c.a0 > lead ? c.a0 - lead : 0u;
  c.mpos = im.nmk ? first_marker(mk, im.nmk, c.pos, c.midx) : kInf;
  schain_tables(c, im, tabs, mt, acm);
  bw_init(c.b, stream, im.ds_lsw, c.pos);
  c.ev = c.a0 < c.mpos ? c.a0 : c.mpos;
}

// pos >= ev: the lead-in's loop head (marker, end of the lead-in), then, in
// the range, decode_range's event block (marker, checkpoint, end)
template <class TAB>
DG_HD void schain_event(SyncChain<TAB> &c, const ImageDesc &im, const TAB *tabs, const DG_GLOBAL uint8_t *stream,
                        const DG_GLOBAL uint32_t *mk, const uint16_t *mt, uint32_t acm) {
  const uint32_t cbits = im.comp_bits;
  if (c.phase == 0) {
    if (c.pos >= c.mpos) {  // restart marker before the start: exact state from here
      c.pos = c.mpos;
      c.r = 0;
      c.z = 0;
      c.comp = cbits & 3u;
      schain_tables(c, im, tabs, mt, acm);
      c.midx++;
      c.mpos = c.midx < im.nmk ? mk[c.midx] : kInf;
      bw_seek(c.b, c.pos);
    }
    if (c.pos < c.a0) {
      c.ev = c.a0 < c.mpos ? c.a0 : c.mpos;
      return;
    }
    const uint32_t rel = c.pos - c.a0;
    c.in = pack_state(rel > 255 ? 255 : rel, c.r, c.z);
    schain_range(c, im, tabs, stream, mk, mt, acm, false);
    if (c.phase != 1 || c.pos < c.ev) return;
  }
  if (c.phase != 1) return;
  if (c.pos >= c.mpos) {  // restart marker: hard resync
    const bool owned = c.mpos < c.a1;
    c.pos = c.mpos;
    c.r = 0;
    c.z = 0;
    c.comp = cbits & 3u;
    schain_tables(c, im, tabs, mt, acm);
    if (owned) {
      c.acc.m++;
      c.acc.n = 0;
      c.acc.dc[0] = c.acc.dc[1] = c.acc.dc[2] = 0;
    }
    c.midx++;
    c.mpos = c.midx < im.nmk ? mk[c.midx] : kInf;
    bw_seek(c.b, c.pos);
  }
  if (c.k < c.nck && c.cpos < c.a1 && c.pos >= c.cpos) {  // first boundary at/after checkpoint k
    const uint32_t rel = c.pos - c.cpos;
    DG_GLOBAL Ckpt &ck = c.ck[c.k];
    ck.st = pack_state(rel > 255 ? 255 : rel, c.r, c.z);
    ck.m = c.acc.m;
    ck.n = c.acc.n;
    ck.dc[0] = c.acc.dc[0];
    ck.dc[1] = c.acc.dc[1];
    ck.dc[2] = c.acc.dc[2];
    c.k++;
    c.cpos += kCkptBits;
  }
  if (c.pos >= c.a1) {  // the range's end: exit state, checkpoint prefixes -> tails
    const uint32_t rel = c.pos - c.a1;
    c.acc.out = pack_state(rel > 255 ? 255 : rel, c.r, c.z);
    for (uint32_t j = 0; j < c.k; j++) {
      DG_GLOBAL Ckpt &ck = c.ck[j];
      if (c.acc.m > ck.m) {
        ck.m = c.acc.m - ck.m;
        ck.n = c.acc.n;
        ck.dc[0] = c.acc.dc[0];
        ck.dc[1] = c.acc.dc[1];
        ck.dc[2] = c.acc.dc[2];
      } else {
        ck.m = 0;
        ck.n = c.acc.n - ck.n;
        ck.dc[0] = c.acc.dc[0] - ck.dc[0];
        ck.dc[1] = c.acc.dc[1] - ck.dc[1];
        ck.dc[2] = c.acc.dc[2] - ck.dc[2];
      }
    }
    c.phase = 2;
    c.ev = kInf;
    return;
  }
  const uint32_t e = c.a1 < c.mpos ? c.a1 : c.mpos;
  c.ev = (c.k < c.nck && c.cpos < e) ? c.cpos : e;
}

// The per-symbol step of two chains, written as their table reads first
// (four independent LDS lookups) and their state updates after.
template <class TAB>
DG_HD void schain_commit(SyncChain<TAB> &c, const ImageDesc &im, const TAB *tabs, const uint16_t *mt, uint32_t acm,
                         uint32_t bits, uint32_t e, uint32_t m) {
  const bool isdc = c.z == 0u;
  const bool live = c.phase != 2u;
  const uint32_t len = e >> 8, sym = e & 0xFFu;
  const uint32_t size = sym & 15u;
  const int32_t v = huff_value(bits, len, size);
  const uint32_t mc = m & 15u;
  const uint32_t zm = c.pos + mc <= c.ev ? multi_next_z(m, c.z) : 0xFFFFFFFFu;
  const bool take_m = zm != 0xFFFFFFFFu;
  const uint32_t np = c.pos + (take_m ? mc : len + size);
  c.pos = live ? np : c.pos;
  const bool cnt = isdc && live;
  c.acc.n += cnt ? 1u : 0u;
  add3(c.acc.dc, c.comp, cnt ? v : 0);
  const uint32_t zn = take_m ? zm : huff_next_z(c.z, sym);
  bw_shift(c.b, c.pos);
  const bool bend = zn >= 64u;
  c.z = bend ? 0u : zn;
  c.r = bend ? (c.r + 1u == im.bpm ? 0u : c.r + 1u) : c.r;
  c.comp = (im.comp_bits >> (2u * c.r)) & 3u;
  schain_tables(c, im, tabs, mt, acm);
}

template <class TAB>
DG_HD void schain_step2(SyncChain<TAB> &A, SyncChain<TAB> &B, const ImageDesc &im, const TAB *tabs,
                        const uint16_t *mt, uint32_t acm) {
  bw_refill(A.b);
  bw_refill(B.b);
  const uint32_t ba = bw_peek(A.b, A.pos), bb = bw_peek(B.b, B.pos);
  const TAB &ta = *(A.z == 0u ? A.tdc : A.tac), &tb = *(B.z == 0u ? B.tdc : B.tac);
  uint32_t ea = ta.lut[ba >> (32 - kLutBits)], eb = tb.lut[bb >> (32 - kLutBits)];
  const uint32_t ma = (A.mi != 3u && A.z != 0u) ? (uint32_t)mt[(A.mi << kMultiBits) | (ba >> (32u - kMultiBits))] : 0u;
  const uint32_t mb = (B.mi != 3u && B.z != 0u) ? (uint32_t)mt[(B.mi << kMultiBits) | (bb >> (32u - kMultiBits))] : 0u;
  if (ea == 0u || (ea & 0x8000u)) ea = huff_lookup(ta, ba);  // codes longer than the first level
  if (eb == 0u || (eb & 0x8000u)) eb = huff_lookup(tb, bb);
  schain_commit(A, im, tabs, mt, acm, ba, ea, ma);
  schain_commit(B, im, tabs, mt, acm, bb, eb, mb);
}

// Both chains to their ends (lead-in + range each).
template <class TAB>
DG_HD void schain_run2(SyncChain<TAB> &A, SyncChain<TAB> &B, const ImageDesc &im, const TAB *tabs,
                       const DG_GLOBAL uint8_t *stream, const DG_GLOBAL uint32_t *mk, const uint16_t *mt,
                       uint32_t acm) {
  for (;;) {
    if (A.pos >= A.ev) schain_event(A, im, tabs, stream, mk, mt, acm);
    if (B.pos >= B.ev) schain_event(B, im, tabs, stream, mk, mt, acm);
    if (A.phase == 2u && B.phase == 2u) break;
    schain_step2(A, B, im, tabs, mt, acm);
  }
}

// ------------------------------------------------------------ destuffing

// Classify raw byte i of a scan: returns 1 if it carries entropy-coded data,
// sets *marker when it is the FF of an RST marker (FF D0..D7).
//   FF 00 -> FF kept, 00 dropped; FF FF -> first FF is fill (dropped);
//   FF Dn -> both dropped, marker recorded at the FF.
DG_HD uint32_t destuff_keep(uint32_t prev, uint32_t cur, uint32_t next, bool first, uint32_t *marker) {
  *marker = 0;
  if (!first && prev == 0xFF && cur != 0xFF) return 0;  // 00 of a stuffed pair, or the code of a marker
  if (cur == 0xFF) {
    if (next == 0x00) return 1;
    if (next >= 0xD0 && next <= 0xD7) *marker = 1;
    return 0;  // fill byte or marker prefix
  }
  return 1;
}

}  // namespace dg
