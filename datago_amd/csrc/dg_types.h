// dg_types.h — POD structures shared by the host planner and the HIP kernels.
//
// One batch = N images.  The host parses headers (host/jpeg_header.cpp),
// chooses buckets (host/buckets.cpp), lays every per-image buffer out in one
// device arena and uploads an array of ImageDesc + per-kernel workgroup lists
// (WgItem).  All device addresses inside these structs are absolute.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define DG_HD __host__ __device__ __forceinline__
#define DG_DEVICE 1
#define DG_GLOBAL __attribute__((address_space(1)))  // global memory: global_load/store, not flat
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#else
#define DG_HD static inline
#define DG_GLOBAL
#endif

namespace dg {

// Typed pointer to device memory from an address held in a descriptor.
template <class T>
DG_HD DG_GLOBAL T *gp(uint64_t a) {
  return (DG_GLOBAL T *)(uintptr_t)a;
}

// Three per-component counters without dynamic register indexing (which would
// spill to scratch): c in {0,1,2}.
DG_HD int32_t sel3(const int32_t v[3], uint32_t c) { return c == 0 ? v[0] : (c == 1 ? v[1] : v[2]); }
DG_HD void add3(int32_t v[3], uint32_t c, int32_t d) {
  v[0] += c == 0 ? d : 0;
  v[1] += c == 1 ? d : 0;
  v[2] += c == 2 ? d : 0;
}

constexpr int kLutBits = 10;          // Huffman first-level lookup width
constexpr int kMaxSlots = 6;         // Huffman tables per image (DC/AC x 3 components)
constexpr int kSubPerWg = 256;       // entropy subsequences per workgroup (= threads)
constexpr int kDefaultSubBits = 2048; // destuffed bits per subsequence
constexpr int kDestuffChunk = 4096;   // raw bytes per destuff workgroup (256 x 16)
constexpr uint32_t kInf = 0xFFFFFFFFu;

// Canonical Huffman table for the GPU decoder (built on the host, pooled).
// Two-level lookup: the first kLutBits bits index lut[]; codes longer than
// that (JPEG allows 16) continue in a 7-bit subtable selected by the entry.
//   lut entry: (len << 8) | symbol          for codes of length <= kLutBits
//              0x8000 | subtable index      when the prefix starts a long code
//              0                            invalid prefix / fallback below
constexpr int kSubBits = 16 - kLutBits;   // 6
constexpr int kMaxSubTables = 8;
struct HuffTable {
  uint16_t lut[1 << kLutBits];
  uint16_t sub[kMaxSubTables][1 << kSubBits];  // (len << 8) | symbol, 0 = invalid
  uint32_t lim[17];             // fallback (more long prefixes than subtables)
  int32_t valoff[17];
  uint8_t vals[256];
};

struct QuantTable {
  uint16_t q[64];  // natural (row-major) order
};

// Entropy-decoder state at a subsequence boundary:
//   bit 31 valid | bits 16..23 rel (destuffed bits past the anchor) | 8..15 r (block in MCU) | 0..7 z
DG_HD uint32_t pack_state(uint32_t rel, uint32_t r, uint32_t z) {
  return 0x80000000u | (rel << 16) | (r << 8) | z;
}
DG_HD uint32_t st_rel(uint32_t s) { return (s >> 16) & 0xFFu; }
DG_HD uint32_t st_r(uint32_t s) { return (s >> 8) & 0xFFu; }
DG_HD uint32_t st_z(uint32_t s) { return s & 0xFFu; }

// Per-subsequence record (64 bytes).
struct SubState {
  uint32_t in;      // state used at the subsequence start
  uint32_t out;     // state at the first symbol boundary at/after the next anchor
  uint32_t m;       // RST markers owned (FF byte inside this subsequence)
  uint32_t n;       // blocks started after the last owned marker (or the start)
  int32_t dc[3];    // DC differences summed after the last owned marker, per component
  uint32_t seg;     // exclusive segmented scan: restart segment at start
  uint32_t nin;     //   blocks already started in that segment
  int32_t dcin[3];  //   DC predictors at start
  uint32_t nstart;  // decode-once staging: blocks started in the range (all segments)
  uint32_t nent;    //   staged entries
};

enum Colorspace : uint32_t { CS_YCC = 0, CS_RGB = 1, CS_GRAY = 2 };

// Resize pass along one axis (one half of a fast_image_resize `resize` call).
struct ResizePass {
  uint64_t src, dst;        // device addresses
  uint64_t coef;            // int16 [out_size * ksize]   (written by k_coeffs)
  uint64_t bounds;          // int32 {start, size} [out_size] (written by k_coeffs)
  double in0, in1;          // source box along the axis
  uint32_t in_size, out_size;
  uint32_t ksize;           // coefficient slots per output
  int32_t precision;        // written by k_coeffs
  uint32_t src_stride, dst_stride;  // bytes per row
  uint32_t width, rows;     // output extent of this pass (pixels, rows)
  uint32_t out0;            // first output (of out_size) computed: integral crops fold into the pass
  uint32_t bands;           // band H kernel: kHBandRows-row bands per workgroup (option "hb_bands")
  uint32_t row0;            // H pass: first source row; V pass: source row of temp row 0
  uint32_t C;               // channels
  uint32_t kind;            // 0 none, 1 horizontal, 2 vertical
  uint32_t mode;            // H passes: kHFused = source is the YCbCr planes (upsample + colour
                            // in the fill), kHDirect = segment too wide for LDS (legacy kernel)
};
constexpr uint32_t kHFused = 1, kHDirect = 2;
constexpr uint32_t kHVFused = 4;      // pass[0] runs fused with pass[1] in k_resize_hv (its H rows stay in LDS)
// pass[0] of a JPEG runs in k_band_dec (dg_band.hip): IDCT + upsampling + colour + this H pass from the
// coefficients, 16-row strips of kDecCols output columns; kHDecWide: the 640-pixel segment class
constexpr uint32_t kHDecode = 8, kHDecWide = 16;
constexpr uint32_t kDecCols = 128;    // k_band_dec: output columns per workgroup (8 MFMA subtiles of 16)
constexpr uint32_t kDecSeg0 = 320, kDecSeg1 = 640;  // k_band_dec source segment classes (pixels)
constexpr uint32_t kDecStripsDefault = 8;           // k_band_dec: 16-row strips per workgroup (option "dec_strips")
constexpr uint32_t kHVSegPx = 320;    // k_resize_hv: LDS source segment per row (downscales up to ~2.3x)
constexpr uint32_t kHVTapsMax = 24;   // k_resize_hv: V taps (its LDS ring holds 32 rows)
constexpr uint32_t kHVRows = 64;      // k_resize_hv: V output rows per workgroup
constexpr uint32_t kHBandRows = 8;    // rows per workgroup of the band H kernel
constexpr uint32_t kHBandCols = 128;  // output columns per workgroup
constexpr uint32_t kIdctItemStride = 4;  // k_idct_t: L_IDCT items per workgroup (one per wave)

constexpr uint32_t kHSegPx = 640;     // LDS source segment (pixels) per row
constexpr uint32_t kHBandsDefault = 16;  // default ResizePass::bands (8 -> 16: +1.5% overlapped, profiles/r02/bands)

constexpr int kStages = 4;  // R1.H, R1.V, R2.H, R2.V

// ---- PNG (ImageDesc::fmt == kFmtPng)
constexpr uint32_t kFmtJpeg = 0, kFmtPng = 1;
// IDAT payloads are gathered into one contiguous zlib stream (k_png_gather),
// inflated into filtered scanlines (k_png_inflate, one wave per image),
// unfiltered (k_png_unfilter, one wave per 64-row band on a diagonal
// wavefront, consecutive bands pipelined across CUs)
// and, for palette / sub-byte / tRNS images, expanded to 8-bit L/LA/RGB/RGBA
// (k_png_expand).
struct PngDesc {
  uint64_t zs;        // contiguous zlib stream
  uint64_t raw;       // inflated scanlines: height x (1 + rowbytes)
  uint64_t unf;       // unfiltered scanlines (stride ustride); == pix when expand == 0
  uint64_t pal;       // 256 x RGBA palette (device), 0 if none
  uint32_t zlen;      // zlib bytes
  uint32_t rowbytes;  // bytes per scanline (without the filter byte)
  uint32_t ustride;   // stride of unf
  uint32_t bpp;       // filter unit (bytes)
  uint32_t ctype, depth, expand, has_trns;
  uint32_t trns[3];   // gray / RGB transparency key
  uint32_t chunk0;    // chunked inflate: first InfChunk of this image
  uint32_t nchunks;   // 0: serial inflate (small streams)
  uint32_t serial;    // set by the chunked path when the image must be inflated serially
  uint32_t interlace; // Adam7: raw/unf hold the 7 passes back to back (png_adam7_*)
  uint32_t rawlen;    // inflated bytes expected
  uint32_t uf_flag0;  // k_png_unfilter: first band progress flag of this image
};

// Adam7 pass p of a W x H image (PNG spec 8.2): origin (x0, y0), spacing (dx, dy)
DG_HD uint32_t png_a7(uint32_t p, uint32_t k) {
  // x0, y0, dx, dy of the pass, 4 bits each (no table: no scratch on the device)
  const uint32_t t = p == 0 ? 0x8800u : p == 1 ? 0x8804u : p == 2 ? 0x8440u : p == 3 ? 0x4402u
                   : p == 4 ? 0x4220u : p == 5 ? 0x2201u : 0x2110u;
  return (t >> (4 * k)) & 15u;
}
DG_HD void png_adam7_pass(uint32_t W, uint32_t H, uint32_t p, uint32_t &pw, uint32_t &ph) {
  const uint32_t x0 = png_a7(p, 0), y0 = png_a7(p, 1), dx = png_a7(p, 2), dy = png_a7(p, 3);
  pw = W > x0 ? (W - x0 + dx - 1) / dx : 0;
  ph = H > y0 ? (H - y0 + dy - 1) / dy : 0;
}
// Geometry of pass p of an interlaced image: size, unfiltered row bytes and
// 16-byte-aligned stride, offsets of its rows in raw and unf
struct A7Pass {
  uint32_t pw, ph, rb, us;
  uint64_t raw_off, unf_off;
};
DG_HD A7Pass png_adam7(uint32_t W, uint32_t H, uint32_t bitspp, uint32_t p) {
  A7Pass r = {0, 0, 0, 0, 0, 0};
  for (uint32_t q = 0; q <= p; q++) {
    uint32_t pw, ph;
    png_adam7_pass(W, H, q, pw, ph);
    const uint32_t rb = (uint32_t)(((uint64_t)bitspp * pw + 7) / 8), us = (rb + 15) / 16 * 16;
    if (q == p) {
      r.pw = pw;
      r.ph = ph;
      r.rb = rb;
      r.us = us;
    } else if (pw && ph) {
      r.raw_off += (uint64_t)ph * (rb + 1);
      r.unf_off += (uint64_t)ph * us;
    }
  }
  return r;
}

// Chunk-parallel inflate.  The zlib stream of a large PNG is cut into
// chunks of `span` bytes (option "inf_chunk", default kInfChunk).  k_inf_find looks in each chunk (but the first) for
// the first bit position that parses as a dynamic-Huffman block header with
// complete codes; k_inf_decode decodes, one lane per chunk, from there until
// it reaches a block boundary that another chunk starts at (or the end).  A
// match reaching before the chunk's start yields a marker (256 + index into
// the 32 KiB window preceding the chunk); k_inf_resolve walks the chain of
// chunks that the decode proved consistent and writes the bytes.  Anything
// irregular (no candidate chain, overflow, a decode error) sends the image to
// the serial inflate kernel.
constexpr uint32_t kInfChunk = 32768;          // compressed bytes per chunk
constexpr uint32_t kInfCapPerByte = 8;         // output entries per compressed byte of a chunk
constexpr uint32_t kInfNone = 0xFFFFFFFFu;
struct InfChunk {
  uint64_t out;       // uint16 entries: byte value, or 256 + window index
  uint64_t tab;       // per-chunk Huffman tables (k_inf_decode scratch)
  uint32_t image;     // descriptor index
  uint32_t idx;       // chunk index within the image
  uint32_t cap;       // capacity of out (entries)
  uint32_t start;     // bit position of the chunk's first block (kInfNone: no candidate)
  uint32_t len;       // entries produced
  uint32_t stop;      // chunk index whose start the decode reached (nchunks: end of stream)
  uint32_t status;    // 0 ok, 1 decode error, 2 overflow
  uint32_t span;      // compressed bytes per chunk of this image
};
constexpr uint32_t kInfTabBytes = 4096;        // per-chunk table scratch (see k_inf_decode)
// A gather job: copy `len` bytes (one IDAT payload) from src to dst.
struct GatherJob {
  uint64_t src, dst;
  uint32_t len, pad;
};
constexpr uint32_t kGatherPiece = 16384;  // bytes per gather workgroup

// fast_image_resize mul_div_alpha (U8x2 / U8x4): an in-place program over one
// buffer.  prog holds up to three 2-bit ops, lowest first: 1 = multiply
// colour by alpha, 2 = divide by alpha.
struct AlphaOp {
  uint64_t buf;
  uint32_t stride, width, rows, prog;
  uint32_t on_decoded;  // buf is the decoded image (not re-created by a resync round)
  uint32_t pad;
};
constexpr uint32_t kAlphaPoints = 3;  // before call 1, between the calls, after call 2

// ---- JPEG re-encode (pre_encode_images + encode_format jpeg,
// image_processing.rs:374-395): image 0.25's baseline encoder, 1x1 sampling,
// Annex K tables scaled by quality.  Per image: k_enc_fdct (colour + FDCT +
// quantisation per MCU), k_enc_count (bits per block), k_enc_scan (bit
// offsets), k_enc_write (codes OR-ed into a zeroed bit buffer), k_enc_stuff
// (header, 0xFF00 stuffing, padding, EOI).
struct EncTables {
  uint16_t code[4][256];  // DC luma, AC luma, DC chroma, AC chroma
  uint8_t len[4][256];
};
struct EncDesc {
  uint64_t src;        // the transformed image (C channels, row stride src_stride)
  uint64_t coef;       // int16 [nblocks][64], quantised, zigzag order, MCU-interleaved blocks
  uint64_t bits;       // uint32 [nblocks]: bit length of each block -> exclusive bit offsets
  uint64_t words;      // scan bit buffer (stream bytes in memory order), zeroed per batch
  uint64_t out;        // header | stuffed scan | EOI
  uint64_t hdr;        // header bytes (SOI .. SOS)
  uint64_t tab;        // EncTables
  uint32_t src_stride, C, ncomp, mode;  // mode 1: resized LA image read as luma bytes
  uint32_t w, h, nbx, nby;
  uint32_t nblocks, hdr_len, total_bits, enc_bytes;
  uint32_t active, png, pad[2];  // png: PNG re-encode (dg_penc.hip): coef = filtered stream,
                                 // nblocks = 1 KiB pieces, bits = piece bit lengths
  uint64_t aux;                  // png: Adler-32 partials per piece (uint32 x 2)
  uint8_t q[2][64];    // quantisation tables, natural order
};

struct ImageDesc {
  // ---- entropy stream
  uint64_t scan;            // device address of the first raw entropy-coded byte
  uint32_t scan_len;        // raw bytes of entropy-coded data (EOI excluded)
  uint32_t nsub;            // subsequences (sized from the raw length)
  uint32_t sub_base;        // first SubState index
  uint32_t sub_bits;        // bits per subsequence (per image: option "sub_density")
  uint32_t ckpt_base;       // first checkpoint record of this image (nsub * num_ckpt(sub_bits) of them)
  uint64_t ds;              // destuffed stream, word-interleaved (ds_word_index), >= 64 zero bytes past its end
  uint64_t mk;              // RST marker positions in ds (bits), ascending
  uint64_t chunk;           // destuff per-chunk records: uint32 {cnt, mkc, off, mkoff}
  uint32_t nchunk;          // raw chunks of kDestuffChunk bytes
  uint32_t ds_state0;       // k_destuff_one: index of chunk 0's state word (batch-wide, list order)
  uint32_t ds_bits;         // destuffed length in bits (written by k_destuff_scan)
  uint32_t nmk;             // RST markers (written by k_destuff_scan)
  uint32_t slotmap;         // Huffman slot of (component c, dc=0/ac=1) at nibble 2c+ac
  uint32_t mk_cap;          // capacity of the marker list
  uint32_t lead_bits;       // k_huff_sync lead-in before each subsequence (lead_in)
  uint32_t ds_lsw;          // log2(32-bit words per subsequence) of the interleaved stream
  uint32_t ckpt;            // 1: k_huff_sync / k_huff_fix record checkpoints for early merging (option "ckpt")
  uint32_t idct_fused;      // 1: k_huff_write turns completed blocks into plane pixels (option "idct_fused")
  uint32_t stage_cap;       // decode-once: staging capacity per subsequence (groups of 4 entries), 0 = off
  uint32_t restart;         // restart interval (MCUs), 0 = none
  uint32_t blocks_per_seg;  // restart * bpm, 0 = unlimited
  uint32_t total_blocks;
  uint32_t bpm;             // blocks per MCU
  uint32_t comp_bits;       // component of block k within an MCU at bits 2k..2k+1
  uint8_t blk_comp[12];     // same, unpacked (host side / IDCT)
  uint16_t hslot[kMaxSlots];  // pool index of Huffman slot s
  uint8_t ncomp, colorspace, dec_c, nslots;  // dec_c: channels of the decoded image
  uint16_t qpool[3];
  uint16_t sem;             // decode semantics: 0 libjpeg-turbo, 1 zune-jpeg (option "decode_semantics")
  uint64_t coef;            // device address of block 0 (int16 zigzag[64] per block, decode order)
  uint64_t stage;           // decode-once staging (dg_entropy.h StageCtx), 0 = off
  // Sparse coefficient blocks (option "sparse_coef"): one byte per block, the
  // mask of the 16-byte zigzag parts k_huff_write stored (its nonzero ones;
  // 0xFF for a block two ranges share); k_idct_t loads only those parts and
  // takes the rest as zero.  0 = dense blocks (every part written and read).
  uint64_t ccnt;
  // ---- geometry
  uint32_t width, height;
  uint32_t mcux, mcuy;
  uint32_t hmax, vmax;
  uint32_t ch[3], cv[3];    // sampling factors
  uint32_t cfirst[3];       // first block of component c within an MCU
  uint32_t cbw[3], cbh[3];  // plane size in blocks
  uint32_t cdsw[3], cdsh[3];// downsampled width/height (libjpeg downsampled_width)
  uint64_t plane[3];        // device address of component planes (stride cbw*8)
  uint64_t pix;             // decoded interleaved image (stride pix_stride), 0 for gray
  uint32_t pix_stride;
  int32_t status;           // set by kernels on corruption
  // ---- resize plan
  ResizePass pass[kStages];
  uint64_t out;             // final output (tight rows)
  uint32_t out_w, out_h, out_c, out_stride;
  uint64_t final_src;       // copy-kernel source (no pass runs, or gray->RGB expansion)
  uint32_t final_src_stride, copy_needed;
  uint32_t final_src_c;
  uint32_t color_fused;     // 1: pass[0] converts colour itself, pix is never written
  // ---- format, PNG, alpha handling, final conversion
  uint32_t fmt;             // kFmtJpeg / kFmtPng
  uint32_t prog;            // progressive JPEG: scans decoded by k_prog_scan (0: sequential)
  uint32_t crec;            // bit c: component c's plane holds chroma records (dg_plane.h; option "chroma_rec")
  uint32_t copy_mode;       // k_copy: 0 same channels, 1 L->RGB, 2 RGBA->RGB blend over gray,
                            // 3 LA->RGB of a resized LA image (GrayImage over the LA bytes, B3),
                            // 4 LA->RGB of an unresized LumaA8 (alpha dropped)
  PngDesc png;
  AlphaOp aop[kAlphaPoints];
  EncDesc enc;
};

// ---- progressive JPEG (ImageDesc::prog > 0).  The coefficient blocks are
// zeroed (k_prog_zero), then every scan is decoded by one wave of k_prog_scan
// straight from the stuffed bytes.  Scans that touch disjoint (component,
// coefficient band) sets are independent; the host gives each scan a level
// (1 + the highest level of an earlier overlapping scan) and the list of
// those earlier scans (deps).  All scans of a batch run in one launch,
// taken in level order; a scan waits, chunk by chunk, only until its deps
// have written the MCU rows it is about to read (a pipeline over the
// image's rows instead of a barrier per level).
struct ProgScan {
  uint64_t data;        // device address of the scan's first entropy-coded byte
  uint32_t len;         // entropy-coded bytes (up to the next non-RST marker)
  uint32_t image;       // descriptor index
  uint32_t ns;          // components in the scan
  uint32_t comp[4];     // their component indices
  uint16_t dc[4];       // DC-first scans: Huffman pool index per scan component
  uint16_t ac;          // AC scans: Huffman pool index
  uint16_t pflags;      // kProgChained: the scan runs after its deps in the same work item (no waits)
  uint32_t ss, se, ah, al;
  uint32_t restart;     // restart interval (MCUs; blocks when ns == 1), 0 = none
  uint32_t level;
  uint32_t first;       // batch index of the image's first scan
  uint32_t next;        // next scan of the same work item (chain), kProgNoScan = none
  uint64_t deps;        // earlier scans of the image this one reads (bit e = scan first + e)
};
// Pipelined scans (one launch per batch): progress word of scan j =
// flags[1 + j], in MCU rows whose blocks the scan has written (kProgDone
// when finished); flags[0] hands out scans to workgroups in list order.
constexpr uint32_t kProgDone = 0xFFFFFFFFu;
constexpr uint32_t kProgNoScan = 0xFFFFFFFFu;
constexpr uint16_t kProgChained = 1;
constexpr uint32_t kProgMaxScans = 256;    // per image (the parser's limit)
constexpr uint32_t kProgMaxDepScans = 64;  // deps is a 64-bit mask: images with more scans run chained only
constexpr uint32_t kProgZeroBytes = 65536;  // coefficient bytes zeroed per k_prog_zero workgroup

// One workgroup's work: an image and the first item it handles.
struct WgItem {
  uint32_t image;
  uint32_t item0;
};

// Batch-wide flags written by kernels (zeroed before each batch).
struct BatchFlags {
  uint32_t chain_changed;   // k_huff_fix changed a workgroup's last exit state
  uint32_t fix_count;       // workgroups k_huff_fix had to re-run
  uint32_t write_mismatch;  // k_huff_write exit != next subsequence's input
  uint32_t sync_iters_max;  // longest intra-workgroup sync loop
  uint32_t idct_late;       // fused IDCT: blocks k_huff_write left to k_idct_list (entries in idct_list)
  uint32_t png_next;        // k_png_inflate mode 1: next list entry a workgroup claims
  uint64_t wgtime;          // debug: device array of {start, end} s_memrealtime per workgroup, 0 = off
  uint32_t wgtime_write;    // first record of k_huff_write's workgroups
  uint32_t debug;           // test switches (kDbg*), kept across resync rounds
  uint64_t idct_list;       // fused IDCT: uint32 {image, block} pairs, idct_cap of them
  uint32_t idct_cap;
  uint32_t prio;            // option "entropy_prio": wave issue priority of k_huff_sync / k_huff_write (0-3)
};
// The counters a resync round clears (everything before `wgtime`).
constexpr size_t kFlagCounters = 24;
// BatchFlags::debug: force the failure paths a valid stream never takes, so
// tests can check that they surface as a per-image status.
constexpr uint32_t kDbgForceWriteMismatch = 1u;  // k_huff_write: subsequence 0 of every image disagrees
constexpr uint32_t kDbgForceChainChange = 2u;    // k_huff_fix: the chain never settles

}  // namespace dg
