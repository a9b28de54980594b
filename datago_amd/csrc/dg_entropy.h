// dg_entropy.h — self-synchronising parallel Huffman decoding of one JPEG
// entropy-coded segment range (host+device code; the kernels in kernels.hip
// and the CPU emulator in tests/native/ both include it).
//
// A scan is cut into fixed raw-byte subsequences [a_i, a_{i+1}).  The thread
// of subsequence i decodes every symbol whose first bit lies in its range.
// Its entry state (bits to skip past a_i, block-in-MCU r, zigzag index z)
// comes from the exit state of subsequence i-1 ("the first symbol boundary at
// or after a_i"); with a guessed entry it usually falls into step with the
// true decode within a few symbols (Huffman self-synchronisation), so the
// workgroup iterates "re-decode from the predecessor's exit" until no exit
// changes.  Byte stuffing (FF 00) is removed while reading; an RST marker
// (FF D0..D7) is a hard sync point: at the first symbol boundary past it the
// state resets to (r=0, z=0) and the DC predictors reset (T.81 F.2.1.3.1).
// Positions are destuffed bit counts relative to the reader's own start, and
// states cross the boundary relative to the anchor a_{i+1}, which both
// neighbours can locate.
#pragma once
#include "dg_types.h"

namespace dg {

DG_HD int32_t huff_extend(int32_t v, int32_t s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

struct BitReader {
  const uint8_t *d;
  uint32_t p, end, anchor;
  uint32_t anchor_bits;  // destuffed position of the anchor, kInf until the refill passes it
  uint32_t loaded;       // destuffed bits loaded
  uint32_t consumed;     // destuffed bits consumed
  uint32_t mpos, mraw;   // pending RST marker: destuffed position and raw index of its FF
  uint64_t buf;          // left-aligned
  int32_t nb;
  int32_t stop;
};

// Start reading at raw index a (the second byte of a pair that began before a
// belongs to the previous range).
DG_HD void br_init(BitReader &b, const uint8_t *d, uint32_t a, uint32_t end, uint32_t anchor) {
  b.d = d;
  b.p = a;
  if (a > 0 && a < end && d[a - 1] == 0xFF && d[a] != 0xFF) b.p = a + 1;
  b.end = end;
  b.anchor = anchor;
  b.anchor_bits = kInf;
  b.loaded = 0;
  b.consumed = 0;
  b.mpos = kInf;
  b.mraw = kInf;
  b.buf = 0;
  b.nb = 0;
  b.stop = 0;
}

// 8 bytes at an arbitrary address.  Device: two/three aligned dword loads
// (callers guarantee 12 readable bytes past the address and that the buffer
// start is 16-byte aligned); host: memcpy.
DG_HD uint64_t load8(const uint8_t *p) {
#if defined(DG_DEVICE)
  uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3) * 8;
  uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  return sh ? ((lo >> sh) | ((uint64_t)w[2] << (64 - sh))) : lo;
#else
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
#endif
}

DG_HD void br_refill(BitReader &b) {
  while (b.nb <= 56) {
    if (b.anchor_bits == kInf && b.p >= b.anchor) b.anchor_bits = b.loaded;
    if (b.stop || b.mpos != kInf) {  // feed zero bits past a marker / the end (libjpeg)
      b.nb += 8;
      continue;
    }
    if (b.p >= b.end) {
      b.stop = 1;
      if (b.anchor_bits == kInf) b.anchor_bits = b.loaded;
      continue;
    }
    // fast path: next 8 bytes hold no 0xFF -> append up to 4 at once
    if (b.nb <= 24 && b.p + 12 <= b.end) {
      uint64_t v = load8(b.d + b.p);  // little-endian bytes p..p+7
      uint64_t nv = ~v;
      uint64_t hasff = (nv - 0x0101010101010101ull) & ~nv & 0x8080808080808080ull;
      if (!hasff) {
        uint32_t take = 4;  // nb <= 24 leaves room for 32 bits
        if (b.anchor_bits == kInf && b.anchor > b.p && b.anchor - b.p < take) take = b.anchor - b.p;
        for (uint32_t k = 0; k < take; k++) {
          b.buf |= (uint64_t)((v >> (8 * k)) & 0xFF) << (56 - b.nb);
          b.nb += 8;
        }
        b.loaded += 8 * take;
        b.p += take;
        continue;
      }
    }
    uint32_t c = b.d[b.p];
    if (c != 0xFF) {
      b.buf |= (uint64_t)c << (56 - b.nb);
      b.nb += 8;
      b.loaded += 8;
      b.p += 1;
      continue;
    }
    uint32_t nx = (b.p + 1 < b.end) ? b.d[b.p + 1] : 0xD9u;
    if (nx == 0x00) {
      b.buf |= (uint64_t)0xFF << (56 - b.nb);
      b.nb += 8;
      b.loaded += 8;
      b.p += 2;
    } else if (nx == 0xFF) {
      b.p += 1;  // fill byte
    } else if (nx >= 0xD0 && nx <= 0xD7) {
      b.mpos = b.loaded;
      b.mraw = b.p;
      b.p += 2;
    } else {
      b.stop = 1;  // EOI or another marker: end of entropy data
      if (b.anchor_bits == kInf) b.anchor_bits = b.loaded;
    }
  }
}

DG_HD void br_skip(BitReader &b, int32_t k) {
  b.buf <<= k;
  b.nb -= k;
  b.consumed += (uint32_t)k;
}

DG_HD int32_t br_get(BitReader &b, int32_t k) {
  if (k == 0) return 0;
  int32_t v = (int32_t)(b.buf >> (64 - k));
  br_skip(b, k);
  return v;
}

template <class T>
DG_HD int32_t huff_decode(BitReader &b, const T &t) {
  uint32_t pk = (uint32_t)(b.buf >> 48);
  uint32_t e = t.lut[pk >> (16 - kLutBits)];
  int32_t len, sym;
  if (e) {
    len = (int32_t)(e >> 8);
    sym = (int32_t)(e & 0xFF);
  } else {
    len = 16;
    sym = 0;  // invalid code: consume 16 bits (only reachable off-sync / past the data)
    for (int32_t l = kLutBits + 1; l <= 16; l++) {
      if (pk < t.lim[l]) {
        len = l;
        sym = t.vals[(t.valoff[l] + (int32_t)(pk >> (16 - l))) & 255];
        break;
      }
    }
  }
  br_skip(b, len);
  return sym;
}

// Accumulators of one subsequence decode.
struct RangeAcc {
  uint32_t out;
  uint32_t m, n;
  int32_t dc[3];
};

// Write-side context (only used when WRITE): coefficient block buffer of this
// thread (64 int16, zigzag order), global coefficient base, prefix values.
struct WriteCtx {
  int16_t *blk;      // thread-private 64-entry buffer
  int16_t *coef;     // image block 0
  uint32_t seg, nin;
  int32_t pred[3];
  uint32_t blocks_per_seg, total_blocks;
  int32_t cur;       // global block index of the block being filled (-1 = none/invalid)
  uint32_t zs;       // first zigzag index this thread owns in the current block
};

DG_HD int32_t wc_index(const WriteCtx &w, uint32_t in_seg) {
  if (w.blocks_per_seg && in_seg >= w.blocks_per_seg) return -1;
  uint64_t g = (uint64_t)(w.blocks_per_seg ? w.seg : 0) * w.blocks_per_seg + in_seg;
  return g < w.total_blocks ? (int32_t)g : -1;
}

DG_HD void wc_begin(WriteCtx &w, int32_t idx, uint32_t zs) {
  w.cur = idx;
  w.zs = zs;
  for (int i = 0; i < 64; i++) w.blk[i] = 0;
}

DG_HD void wc_flush(WriteCtx &w, uint32_t ze) {
  if (w.cur < 0) return;
  int16_t *dst = w.coef + (size_t)w.cur * 64;
  if (w.zs == 0 && ze == 64) {
#if defined(DG_DEVICE)
    const uint4 *s4 = (const uint4 *)w.blk;
    uint4 *d4 = (uint4 *)dst;
#pragma unroll
    for (int i = 0; i < 8; i++) d4[i] = s4[i];
#else
    for (int i = 0; i < 64; i++) dst[i] = w.blk[i];
#endif
  } else {
    for (uint32_t i = w.zs; i < ze; i++) dst[i] = w.blk[i];
  }
  w.cur = -1;
}

// Decode the symbols of subsequence `s` of image `im` starting from `in`.
// tabs: Huffman tables indexed by slot (dc_slot/ac_slot of the image).
template <bool WRITE, class TAB>
DG_HD void decode_range(const ImageDesc &im, const TAB *tabs, const uint8_t *scan, uint32_t s,
                        uint32_t in, RangeAcc &acc, WriteCtx *w) {
  uint32_t a0 = s * im.sub_bytes;
  uint32_t a1 = (s + 1 == im.nsub) ? im.scan_len : a0 + im.sub_bytes;
  BitReader b;
  br_init(b, scan, a0, im.scan_len, a1);
  uint32_t r = st_r(in), z = st_z(in);
  const uint32_t bpm = im.bpm;
  acc.m = 0;
  acc.n = 0;
  acc.dc[0] = acc.dc[1] = acc.dc[2] = 0;
  br_refill(b);
  br_skip(b, (int32_t)st_rel(in));
  uint32_t comp = im.blk_comp[r];
  if (WRITE) {
    w->cur = -1;
    if (z > 0) wc_begin(*w, w->nin > 0 ? wc_index(*w, w->nin - 1) : -1, z);
  }
  for (;;) {
    if (b.consumed >= b.mpos) {  // restart marker reached: hard resync
      bool owned = b.mraw < a1;
      if (WRITE && z > 0) wc_flush(*w, z);
      b.consumed = b.mpos;
      b.buf = 0;
      b.nb = 0;
      b.mpos = kInf;
      r = 0;
      z = 0;
      comp = im.blk_comp[0];
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
    }
    br_refill(b);
    if (b.anchor_bits != kInf && b.consumed >= b.anchor_bits) break;
    if (z == 0) {
      const TAB &t = tabs[im.dc_slot[comp]];
      int32_t sc = huff_decode(b, t) & 15;
      int32_t diff = sc ? huff_extend(br_get(b, sc), sc) : 0;
      acc.n++;
      acc.dc[comp] += diff;
      z = 1;
      if (WRITE) {
        w->pred[comp] += diff;
        wc_begin(*w, wc_index(*w, w->nin), 0);
        w->nin++;
        w->blk[0] = (int16_t)w->pred[comp];
      }
    } else {
      const TAB &t = tabs[im.ac_slot[comp]];
      int32_t rs = huff_decode(b, t);
      int32_t run = rs >> 4, sz = rs & 15;
      if (sz) {
        z += (uint32_t)run;
        int32_t v = huff_extend(br_get(b, sz), sz);
        if (WRITE && z < 64) w->blk[z] = (int16_t)v;
        z++;
      } else if (run == 15) {
        z += 16;
      } else {
        z = 64;
      }
      if (z >= 64) {
        if (WRITE) wc_flush(*w, 64);
        z = 0;
        r = (r + 1 == bpm) ? 0 : r + 1;
        comp = im.blk_comp[r];
      }
    }
  }
  if (WRITE && z > 0) wc_flush(*w, z);
  uint32_t rel = b.consumed - b.anchor_bits;
  acc.out = pack_state(rel > 255 ? 255 : rel, r, z);
}

}  // namespace dg
