/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's library; the product path
 * (datago_amd/csrc) never links or calls it.
 *
 * A plain-C, scalar restatement of baseline/extended-sequential and
 * progressive Huffman JPEG decoding, written from ITU-T T.81 and following
 * libjpeg-turbo's decompression semantics (the decoder PIL uses in this image):
 *   - Huffman decode + HUFF_EXTEND per T.81 F.2.2 (libjpeg jdhuff.c),
 *   - progressive scans per T.81 G.1.2 (libjpeg jdphuff.c: DC first/refine,
 *     AC first with EOB runs, AC refine with correction bits); files whose
 *     coefficients 1..9 stay incomplete after the last scan (libjpeg would
 *     apply block smoothing, jdcoefct.c smoothing_ok) are UNSUPPORTED
 *     (under OJ_SEM_ZUNE they decode as they stand: zune-jpeg does not smooth),
 *   - ISLOW integer IDCT (libjpeg jidctint.c, CONST_BITS=13, PASS1_BITS=2) with
 *     the SIMD build's saturating output (clamp to [-128,127] + 128),
 *   - "fancy" triangular chroma upsampling h2v1 / h2v2 (libjpeg jdsample.c),
 *     with box replication when downsampled_width <= 2, edge rows/columns
 *     replicated,
 *   - YCbCr->RGB with libjpeg's 16-bit fixed-point tables (jdcolor.c),
 *   - colour-space guess from JFIF/Adobe markers and component ids
 *     (libjpeg jdapimin.c default_decompress_parms).
 *
 * Where it stands relative to the reference: datago decodes JPEG through
 * `image 0.25.9` -> `zune-jpeg 0.5.12` (reference worker_files.rs:8-17,
 * worker_wds.rs:45, worker_http.rs:64; pinned in Cargo.lock).  That crate is
 * not vendored under /root/reference and no Rust toolchain exists here, so the
 * decoded pixel values of the reference are UNPINNED; this oracle is instead
 * pinned bit-exactly against PIL/libjpeg-turbo 3.1 (tests/test_oracle_jpeg.py
 * and the committed fixtures in tests/golden/).
 *
 * Decode semantics switch (oj_set_semantics, SURVEY Appendix B: "encode each
 * behind a single switch"): OJ_SEM_LIBJPEG (default, above, pinned) or
 * OJ_SEM_ZUNE, a restatement of zune-jpeg 0.5.12's pixel stages as published
 * in its source (recalled; the crate is not vendored, so this mode is
 * PARITY UNPINNED):
 *   - IDCT `idct_int` (zune-jpeg src/idct/scalar.rs; its AVX2 twin is
 *     lane-for-lane the same): stb_image's integer IDCT, 12-bit constants,
 *     pass 1 (x + 512) >> 10, pass 2 (x + 65536 + (128 << 17)) >> 17, clamped
 *     to 0..255,
 *   - upsampling (src/upsampler/scalar.rs) over the MCU-padded component
 *     rows: horizontal (3*a + b + 2) >> 2 on both output phases, first output
 *     = in[0], last pair from in[n-2], in[n-1]; vertical (h2v2) first
 *     (3*cur + near + 2) >> 2 then horizontal on each output row; the row
 *     above the first / below the last padded row is the row itself,
 *   - YCbCr->RGB (src/color_convert/scalar.rs): r = y + (45*cr' >> 5),
 *     g = y - ((11*cb' + 23*cr') >> 5), b = y + (113*cb' >> 6) with
 *     cb' = cb - 128, cr' = cr - 128, clamped.
 * Entropy decoding and dequantisation are format-defined and identical in
 * both modes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OJ_SEM_LIBJPEG 0
#define OJ_SEM_ZUNE 1
static int g_sem = OJ_SEM_LIBJPEG;
void oj_set_semantics(int s) { g_sem = s == OJ_SEM_ZUNE ? OJ_SEM_ZUNE : OJ_SEM_LIBJPEG; }
int oj_get_semantics(void) { return g_sem; }

#define OJ_OK 0
#define OJ_UNSUPPORTED 1
#define OJ_CORRUPT 2
#define OJ_SMALLBUF 3

static const int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63,
    /* extra entries for safety against corrupt run lengths (libjpeg does the same) */
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct {
  int present;
  uint8_t bits[17];
  uint8_t vals[256];
  int32_t mincode[17];
  int32_t maxcode[18];
  int32_t valptr[17];
} oj_huff;

typedef struct {
  int id, h, v, tq, td, ta;
  int dsw, dsh;        /* downsampled_width/height: ceil(W*h/hmax), ceil(H*v/vmax) */
  int bw, bh;          /* blocks per line / block rows allocated */
  int16_t *coef;       /* bw*bh*64, natural order, quantized */
  uint8_t *plane;      /* (bw*8) x (bh*8) */
} oj_comp;

typedef struct {
  int W, H, ncomp, precision, sof;
  int hmax, vmax, mcux, mcuy;
  int restart;
  int jfif, adobe, adobe_transform;
  uint16_t q[4][64];
  int qpresent[4];
  oj_huff dc[4], ac[4];
  oj_comp comp[4];
  int scan_ncomp;
  int scan_comp[4];
  size_t scan_off;     /* offset of the first entropy-coded byte */
  int saw_sof, saw_sos;
  int progressive;
  int ss, se, ah, al;  /* spectral selection / successive approximation of the current scan */
} oj_jpeg;

#define OJ_EOI 100 /* parse_markers reached EOI (internal) */

/* ---------------------------------------------------------------- markers */

static int build_huff(oj_huff *t) {
  /* canonical code assignment, T.81 Annex C / libjpeg jdhuff.c */
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    t->valptr[l] = k;
    t->mincode[l] = code;
    code += t->bits[l];
    k += t->bits[l];
    t->maxcode[l] = t->bits[l] ? code - 1 : -1;
    if (code > (1 << l)) return OJ_CORRUPT;
    code <<= 1;
  }
  t->maxcode[17] = 0x7fffffff;
  if (k > 256) return OJ_CORRUPT;
  t->present = 1;
  return OJ_OK;
}

static int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

/* Process markers from offset p up to the next SOS (OJ_OK, scan fields set)
 * or EOI (OJ_EOI). */
static int parse_markers(oj_jpeg *j, const uint8_t *d, size_t n, size_t p) {
  for (;;) {
    /* find marker */
    while (p < n && d[p] != 0xFF) p++;
    while (p < n && d[p] == 0xFF) p++;
    if (p >= n) return OJ_CORRUPT;
    int m = d[p++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return OJ_EOI;
    if (p + 2 > n) return OJ_CORRUPT;
    int L = rd16(d + p);
    if (L < 2 || p + L > n) return OJ_CORRUPT;
    const uint8_t *s = d + p + 2;
    int len = L - 2;
    switch (m) {
      case 0xC0: case 0xC1: /* baseline / extended sequential Huffman */
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF: {
        if (m != 0xC0 && m != 0xC1 && m != 0xC2) return OJ_UNSUPPORTED;
        if (len < 6) return OJ_CORRUPT;
        if (j->saw_sof) return OJ_CORRUPT; /* second SOF */
        j->sof = m;
        j->progressive = (m == 0xC2);
        j->precision = s[0];
        j->H = rd16(s + 1);
        j->W = rd16(s + 3);
        j->ncomp = s[5];
        if (j->precision != 8) return OJ_UNSUPPORTED;
        if (j->W == 0 || j->H == 0) return OJ_CORRUPT;
        if (j->ncomp != 1 && j->ncomp != 3) return OJ_UNSUPPORTED;
        if (len < 6 + 3 * j->ncomp) return OJ_CORRUPT;
        for (int c = 0; c < j->ncomp; c++) {
          j->comp[c].id = s[6 + 3 * c];
          j->comp[c].h = s[7 + 3 * c] >> 4;
          j->comp[c].v = s[7 + 3 * c] & 15;
          j->comp[c].tq = s[8 + 3 * c];
          if (j->comp[c].h < 1 || j->comp[c].h > 4 || j->comp[c].v < 1 || j->comp[c].v > 4 ||
              j->comp[c].tq > 3)
            return OJ_CORRUPT;
        }
        j->saw_sof = 1;
        break;
      }
      case 0xC4: { /* DHT */
        int o = 0;
        while (o < len) {
          if (o + 17 > len) return OJ_CORRUPT;
          int tc = s[o] >> 4, th = s[o] & 15;
          if (tc > 1 || th > 3) return OJ_CORRUPT;
          oj_huff *t = tc ? &j->ac[th] : &j->dc[th];
          int total = 0;
          t->bits[0] = 0;
          for (int i = 1; i <= 16; i++) { t->bits[i] = s[o + i]; total += s[o + i]; }
          if (total > 256 || o + 17 + total > len) return OJ_CORRUPT;
          memcpy(t->vals, s + o + 17, (size_t)total);
          if (build_huff(t)) return OJ_CORRUPT;
          o += 17 + total;
        }
        break;
      }
      case 0xDB: { /* DQT */
        int o = 0;
        while (o < len) {
          int pq = s[o] >> 4, tq = s[o] & 15;
          if (tq > 3 || pq > 1) return OJ_CORRUPT;
          if (o + 1 + 64 * (pq + 1) > len) return OJ_CORRUPT;
          for (int k = 0; k < 64; k++)
            j->q[tq][kNatural[k]] = pq ? (uint16_t)rd16(s + o + 1 + 2 * k) : s[o + 1 + k];
          j->qpresent[tq] = 1;
          o += 1 + 64 * (pq + 1);
        }
        break;
      }
      case 0xDD: /* DRI */
        if (len < 2) return OJ_CORRUPT;
        j->restart = rd16(s);
        break;
      case 0xE0: /* APP0: JFIF */
        if (len >= 5 && !memcmp(s, "JFIF\0", 5)) j->jfif = 1;
        break;
      case 0xEE: /* APP14: Adobe */
        if (len >= 12 && !memcmp(s, "Adobe", 5)) { j->adobe = 1; j->adobe_transform = s[11]; }
        break;
      case 0xDA: { /* SOS */
        if (!j->saw_sof) return OJ_CORRUPT;
        int ns = s[0];
        if (ns < 1 || ns > 4 || len < 1 + 2 * ns + 3) return OJ_CORRUPT;
        j->scan_ncomp = ns;
        for (int i = 0; i < ns; i++) {
          int cid = s[1 + 2 * i], c;
          for (c = 0; c < j->ncomp; c++) if (j->comp[c].id == cid) break;
          if (c == j->ncomp) return OJ_CORRUPT;
          j->scan_comp[i] = c;
          j->comp[c].td = s[2 + 2 * i] >> 4;
          j->comp[c].ta = s[2 + 2 * i] & 15;
          if (j->comp[c].td > 3 || j->comp[c].ta > 3) return OJ_CORRUPT;
        }
        int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahal = s[3 + 2 * ns];
        j->ss = ss;
        j->se = se;
        j->ah = ahal >> 4;
        j->al = ahal & 15;
        if (j->progressive) {
          /* libjpeg jdphuff.c start_pass_phuff_decoder: bad progression -> error */
          if (ss == 0) {
            if (se != 0) return OJ_CORRUPT;
          } else {
            if (se < ss || se > 63 || ns != 1) return OJ_CORRUPT;
          }
          if (j->ah != 0 && j->al != j->ah - 1) return OJ_CORRUPT;
          if (j->al > 13) return OJ_CORRUPT;
        } else {
          if (ss != 0 || se != 63 || ahal != 0) return OJ_CORRUPT;
          /* only single-scan sequential images are in scope (all components interleaved) */
          if (ns != j->ncomp) return OJ_UNSUPPORTED;
        }
        j->scan_off = p + L;
        j->saw_sos = 1;
        return OJ_OK;
      }
      default:
        break;
    }
    p += L;
  }
}

static int parse_headers(oj_jpeg *j, const uint8_t *d, size_t n) {
  memset(j, 0, sizeof(*j));
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return OJ_CORRUPT;
  int st = parse_markers(j, d, n, 2);
  return st == OJ_EOI ? OJ_CORRUPT : st; /* EOI before SOS */
}

/* ---------------------------------------------------------- bit reader */

typedef struct {
  const uint8_t *d;
  size_t n, p;
  uint64_t buf;
  int nbits;
  int marker_hit;
} oj_bits;

static void fill(oj_bits *b) {
  while (b->nbits <= 56) {
    uint32_t c = 0;
    if (!b->marker_hit && b->p < b->n) {
      c = b->d[b->p];
      if (c == 0xFF) {
        /* skip fill bytes; 0xFF00 is a stuffed data byte */
        size_t q = b->p + 1;
        while (q < b->n && b->d[q] == 0xFF) q++;
        if (q < b->n && b->d[q] == 0x00) {
          b->p = q + 1;
        } else {
          b->marker_hit = 1; /* marker: feed zeros (libjpeg behaviour); p stays on it */
          c = 0;
        }
      } else {
        b->p++;
      }
    }
    b->buf |= (uint64_t)c << (56 - b->nbits);
    b->nbits += 8;
  }
}

static inline int getbits(oj_bits *b, int k) {
  if (k == 0) return 0;
  if (b->nbits < k) fill(b);
  int v = (int)(b->buf >> (64 - k));
  b->buf <<= k;
  b->nbits -= k;
  return v;
}

/* Huffman symbols decoded since the last reset (tools/entropy_per_symbol.py:
 * instructions per symbol of the GPU entropy kernels). */
static unsigned long long g_symbols = 0;
unsigned long long oj_symbol_count(void) { return g_symbols; }
void oj_reset_symbol_count(void) { g_symbols = 0; }

static inline int decode_sym(oj_bits *b, const oj_huff *t) {
  g_symbols++;
  if (b->nbits < 16) fill(b);
  int code = 0;
  for (int l = 1; l <= 16; l++) {
    code = (code << 1) | (int)(b->buf >> 63);
    b->buf <<= 1;
    b->nbits--;
    if (code <= t->maxcode[l]) return t->vals[(t->valptr[l] + code - t->mincode[l]) & 255];
  }
  return -1; /* corrupt */
}

static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

/* restart: discard buffered bits, consume the RSTn marker (libjpeg
 * jdhuff.c process_restart + jdmarker.c read_restart_marker for well-formed
 * streams). */
static void restart_reader(oj_bits *b) {
  b->buf = 0;
  b->nbits = 0;
  size_t q = b->p;
  while (q + 1 < b->n && !(b->d[q] == 0xFF && b->d[q + 1] >= 0xD0 && b->d[q + 1] <= 0xD7)) q++;
  if (q + 1 < b->n) b->p = q + 2;
  b->marker_hit = 0;
}

static int decode_block(oj_bits *b, const oj_huff *dc, const oj_huff *ac, int *pred, int16_t *blk) {
  int s = decode_sym(b, dc);
  if (s < 0 || s > 15) return OJ_CORRUPT;
  int diff = s ? extend(getbits(b, s), s) : 0;
  *pred += diff;
  blk[0] = (int16_t)*pred;
  for (int k = 1; k < 64; k++) {
    int rs = decode_sym(b, ac);
    if (rs < 0) return OJ_CORRUPT;
    int r = rs >> 4;
    s = rs & 15;
    if (s) {
      k += r;
      int v = extend(getbits(b, s), s);
      blk[kNatural[k]] = (int16_t)v;
    } else {
      if (r != 15) break;
      k += 15;
    }
  }
  return OJ_OK;
}

/* ----------------------------------------------------------- allocation */

static void free_jpeg(oj_jpeg *j) {
  for (int c = 0; c < 4; c++) {
    free(j->comp[c].coef);
    free(j->comp[c].plane);
    j->comp[c].coef = NULL;
    j->comp[c].plane = NULL;
  }
}

static int setup_geometry(oj_jpeg *j) {
  j->hmax = j->vmax = 1;
  for (int c = 0; c < j->ncomp; c++) {
    if (j->comp[c].h > j->hmax) j->hmax = j->comp[c].h;
    if (j->comp[c].v > j->vmax) j->vmax = j->comp[c].v;
  }
  j->mcux = (j->W + 8 * j->hmax - 1) / (8 * j->hmax);
  j->mcuy = (j->H + 8 * j->vmax - 1) / (8 * j->vmax);
  for (int c = 0; c < j->ncomp; c++) {
    oj_comp *k = &j->comp[c];
    k->dsw = (int)(((long)j->W * k->h + j->hmax - 1) / j->hmax);
    k->dsh = (int)(((long)j->H * k->v + j->vmax - 1) / j->vmax);
    if (j->ncomp == 1) {
      k->bw = (k->dsw + 7) / 8;
      k->bh = (k->dsh + 7) / 8;
    } else {
      k->bw = j->mcux * k->h;
      k->bh = j->mcuy * k->v;
    }
    k->coef = (int16_t *)calloc((size_t)k->bw * k->bh * 64, sizeof(int16_t));
    k->plane = (uint8_t *)malloc((size_t)k->bw * 8 * k->bh * 8);
    if (!k->coef || !k->plane) return OJ_SMALLBUF;
    if (!j->qpresent[k->tq]) return OJ_CORRUPT;
    if (!j->progressive && (!j->dc[k->td].present || !j->ac[k->ta].present)) return OJ_CORRUPT;
  }
  return OJ_OK;
}

static int decode_scan(oj_jpeg *j, const uint8_t *d, size_t n) {
  oj_bits b = {d, n, j->scan_off, 0, 0, 0};
  int pred[4] = {0, 0, 0, 0};
  int since_restart = 0;
  if (j->ncomp == 1) {
    oj_comp *k = &j->comp[0];
    int bx_n = (k->dsw + 7) / 8, by_n = (k->dsh + 7) / 8;
    for (int by = 0; by < by_n; by++)
      for (int bx = 0; bx < bx_n; bx++) {
        if (j->restart && since_restart == j->restart) {
          restart_reader(&b);
          pred[0] = 0;
          since_restart = 0;
        }
        int16_t *blk = k->coef + ((size_t)by * k->bw + bx) * 64;
        if (decode_block(&b, &j->dc[k->td], &j->ac[k->ta], &pred[0], blk)) return OJ_CORRUPT;
        since_restart++;
      }
    return OJ_OK;
  }
  for (int my = 0; my < j->mcuy; my++)
    for (int mx = 0; mx < j->mcux; mx++) {
      if (j->restart && since_restart == j->restart) {
        restart_reader(&b);
        memset(pred, 0, sizeof(pred));
        since_restart = 0;
      }
      for (int i = 0; i < j->scan_ncomp; i++) {
        int c = j->scan_comp[i];
        oj_comp *k = &j->comp[c];
        for (int v = 0; v < k->v; v++)
          for (int h = 0; h < k->h; h++) {
            int by = my * k->v + v, bx = mx * k->h + h;
            int16_t *blk = k->coef + ((size_t)by * k->bw + bx) * 64;
            if (decode_block(&b, &j->dc[k->td], &j->ac[k->ta], &pred[c], blk)) return OJ_CORRUPT;
          }
      }
      since_restart++;
    }
  return OJ_OK;
}

/* ------------------------------------------------------- progressive scans */

/* Block (bx, by) of component c in a non-interleaved scan covers the
 * component's ceil(dsw/8) x ceil(dsh/8) blocks (libjpeg jdinput.c
 * per_scan_setup); interleaved scans walk MCUs like the sequential scan. */
typedef struct {
  int eobrun;
  int pred[4];
} oj_pstate;

static int prog_block(oj_jpeg *j, oj_bits *b, oj_pstate *ps, int ci, int16_t *blk) {
  const int ss = j->ss, se = j->se, ah = j->ah, al = j->al;
  oj_comp *k = &j->comp[j->scan_comp[ci]];
  if (ss == 0) {
    if (ah == 0) { /* DC first: jdphuff.c decode_mcu_DC_first */
      int s = decode_sym(b, &j->dc[k->td]);
      if (s < 0 || s > 15) return OJ_CORRUPT;
      int diff = s ? extend(getbits(b, s), s) : 0;
      ps->pred[ci] += diff;
      blk[0] = (int16_t)((uint32_t)ps->pred[ci] << al);
    } else { /* DC refine: decode_mcu_DC_refine */
      if (getbits(b, 1)) blk[0] = (int16_t)(blk[0] | (1 << al));
    }
    return OJ_OK;
  }
  const oj_huff *ac = &j->ac[k->ta];
  if (ah == 0) { /* AC first: decode_mcu_AC_first */
    if (ps->eobrun > 0) {
      ps->eobrun--;
      return OJ_OK;
    }
    for (int kk = ss; kk <= se; kk++) {
      int rs = decode_sym(b, ac);
      if (rs < 0) return OJ_CORRUPT;
      int r = rs >> 4, s = rs & 15;
      if (s) {
        kk += r;
        int v = extend(getbits(b, s), s);
        blk[kNatural[kk]] = (int16_t)((uint32_t)v << al);
      } else if (r == 15) {
        kk += 15;
      } else {
        ps->eobrun = 1 << r;
        if (r) ps->eobrun += getbits(b, r);
        ps->eobrun--;
        break;
      }
    }
    return OJ_OK;
  }
  /* AC refine: decode_mcu_AC_refine */
  const int p1 = 1 << al, m1 = -(1 << al);
  int kk = ss;
  if (ps->eobrun == 0) {
    for (; kk <= se; kk++) {
      int rs = decode_sym(b, ac);
      if (rs < 0) return OJ_CORRUPT;
      int r = rs >> 4, s = rs & 15;
      if (s) {
        s = getbits(b, 1) ? p1 : m1; /* size must be 1 (a warning in libjpeg otherwise) */
      } else if (r != 15) {
        ps->eobrun = 1 << r;
        if (r) ps->eobrun += getbits(b, r);
        break; /* the rest of the block is handled by the EOB run below */
      }
      /* advance over already-nonzero coefficients (appending correction bits)
       * and r still-zero ones */
      do {
        int16_t *c = &blk[kNatural[kk]];
        if (*c != 0) {
          if (getbits(b, 1) && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
        } else {
          if (--r < 0) break; /* reached the target zero coefficient */
        }
        kk++;
      } while (kk <= se);
      if (s) blk[kNatural[kk]] = (int16_t)s;
    }
  }
  if (ps->eobrun > 0) {
    /* scan the rest of the band for correction bits of nonzero coefficients */
    for (; kk <= se; kk++) {
      int16_t *c = &blk[kNatural[kk]];
      if (*c != 0 && getbits(b, 1) && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
    }
    ps->eobrun--;
  }
  return OJ_OK;
}

/* Decode the current progressive scan; *end = reader position afterwards. */
static int prog_scan(oj_jpeg *j, const uint8_t *d, size_t n, size_t *end) {
  oj_bits b = {d, n, j->scan_off, 0, 0, 0};
  oj_pstate ps;
  memset(&ps, 0, sizeof(ps));
  int since_restart = 0;
  /* tables the scan needs */
  for (int i = 0; i < j->scan_ncomp; i++) {
    oj_comp *k = &j->comp[j->scan_comp[i]];
    if (j->ss == 0 && j->ah == 0 && !j->dc[k->td].present) return OJ_CORRUPT;
    if (j->ss > 0 && !j->ac[k->ta].present) return OJ_CORRUPT;
  }
  if (j->scan_ncomp == 1) {
    oj_comp *k = &j->comp[j->scan_comp[0]];
    int bx_n = (k->dsw + 7) / 8, by_n = (k->dsh + 7) / 8;
    for (int by = 0; by < by_n; by++)
      for (int bx = 0; bx < bx_n; bx++) {
        if (j->restart && since_restart == j->restart) {
          restart_reader(&b);
          memset(&ps, 0, sizeof(ps));
          since_restart = 0;
        }
        if (prog_block(j, &b, &ps, 0, k->coef + ((size_t)by * k->bw + bx) * 64)) return OJ_CORRUPT;
        since_restart++;
      }
  } else {
    for (int my = 0; my < j->mcuy; my++)
      for (int mx = 0; mx < j->mcux; mx++) {
        if (j->restart && since_restart == j->restart) {
          restart_reader(&b);
          memset(&ps, 0, sizeof(ps));
          since_restart = 0;
        }
        for (int i = 0; i < j->scan_ncomp; i++) {
          oj_comp *k = &j->comp[j->scan_comp[i]];
          for (int v = 0; v < k->v; v++)
            for (int h = 0; h < k->h; h++) {
              int by = my * k->v + v, bx = mx * k->h + h;
              if (prog_block(j, &b, &ps, i, k->coef + ((size_t)by * k->bw + bx) * 64)) return OJ_CORRUPT;
            }
        }
        since_restart++;
      }
  }
  *end = b.p;
  return OJ_OK;
}

/* Every scan of a progressive file, then the completeness check. */
static int decode_progressive(oj_jpeg *j, const uint8_t *d, size_t n) {
  int bits[4][64];
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 64; k++) bits[c][k] = -1;
  for (;;) {
    for (int i = 0; i < j->scan_ncomp; i++)
      for (int k = j->ss; k <= j->se; k++) bits[j->scan_comp[i]][k] = j->al;
    size_t end;
    int st = prog_scan(j, d, n, &end);
    if (st) return st;
    /* the scan's data ends at the first marker that is not RSTn */
    size_t q = end < j->scan_off ? j->scan_off : end;
    while (q + 1 < n && !(d[q] == 0xFF && d[q + 1] != 0x00 && d[q + 1] != 0xFF && !(d[q + 1] >= 0xD0 && d[q + 1] <= 0xD7)))
      q++;
    if (q + 1 >= n) return OJ_CORRUPT; /* no EOI */
    st = parse_markers(j, d, n, q);
    if (st == OJ_EOI) break;
    if (st) return st;
  }
  if (g_sem == OJ_SEM_ZUNE) return OJ_OK; /* zune-jpeg has no block smoothing: coefficients as decoded */
  for (int c = 0; c < j->ncomp; c++) {
    if (bits[c][0] != 0) return OJ_UNSUPPORTED; /* DC incomplete */
    for (int k = 1; k < 10; k++)
      if (bits[c][k] != 0) return OJ_UNSUPPORTED; /* libjpeg would smooth blocks */
  }
  return OJ_OK;
}

/* ------------------------------------------------------------- ISLOW IDCT */

#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX_0_298631336 ((int32_t)2446)
#define FIX_0_390180644 ((int32_t)3196)
#define FIX_0_541196100 ((int32_t)4433)
#define FIX_0_765366865 ((int32_t)6270)
#define FIX_0_899976223 ((int32_t)7373)
#define FIX_1_175875602 ((int32_t)9633)
#define FIX_1_501321110 ((int32_t)12299)
#define FIX_1_847759065 ((int32_t)15137)
#define FIX_1_961570560 ((int32_t)16069)
#define FIX_2_053119869 ((int32_t)16819)
#define FIX_2_562915447 ((int32_t)20995)
#define FIX_3_072711026 ((int32_t)25172)
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

/* pass-1 workspace values saturate to 16 bits, as in libjpeg-turbo's SIMD
 * IDCTs (vpackssdw between the passes); valid blocks never come near it */
static inline int32_t sat16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

static inline uint8_t clamp_out(int32_t x) {
  /* libjpeg-turbo SIMD IDCT output: saturate to signed 8 bits, then +128 */
  if (x < -128) x = -128;
  if (x > 127) x = 127;
  return (uint8_t)(x + 128);
}

/* one 1-D 8-point ISLOW IDCT; in[i*stride] -> out0..7 (pre-descale sums) */
#define IDCT_1D(i0, i1, i2, i3, i4, i5, i6, i7, o0, o1, o2, o3, o4, o5, o6, o7)             \
  do {                                                                                      \
    int32_t z1, z2, z3, z4, z5, t0, t1, t2, t3, t10, t11, t12, t13;                         \
    z2 = (i2); z3 = (i6);                                                                   \
    z1 = (z2 + z3) * FIX_0_541196100;                                                       \
    t2 = z1 + z3 * (-FIX_1_847759065);                                                      \
    t3 = z1 + z2 * FIX_0_765366865;                                                         \
    z2 = (i0); z3 = (i4);                                                                   \
    t0 = (int32_t)((uint32_t)(z2 + z3) << CONST_BITS);                                      \
    t1 = (int32_t)((uint32_t)(z2 - z3) << CONST_BITS);                                      \
    t10 = t0 + t3; t13 = t0 - t3; t11 = t1 + t2; t12 = t1 - t2;                             \
    t0 = (i7); t1 = (i5); t2 = (i3); t3 = (i1);                                             \
    z1 = t0 + t3; z2 = t1 + t2; z3 = t0 + t2; z4 = t1 + t3;                                 \
    z5 = (z3 + z4) * FIX_1_175875602;                                                       \
    t0 = t0 * FIX_0_298631336; t1 = t1 * FIX_2_053119869;                                   \
    t2 = t2 * FIX_3_072711026; t3 = t3 * FIX_1_501321110;                                   \
    z1 = z1 * (-FIX_0_899976223); z2 = z2 * (-FIX_2_562915447);                             \
    z3 = z3 * (-FIX_1_961570560); z4 = z4 * (-FIX_0_390180644);                             \
    z3 += z5; z4 += z5;                                                                     \
    t0 += z1 + z3; t1 += z2 + z4; t2 += z2 + z3; t3 += z1 + z4;                             \
    o0 = t10 + t3; o7 = t10 - t3; o1 = t11 + t2; o6 = t11 - t2;                             \
    o2 = t12 + t1; o5 = t12 - t1; o3 = t13 + t0; o4 = t13 - t0;                             \
  } while (0)

static void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out, int stride) {
  int32_t ws[64];
  for (int c = 0; c < 8; c++) {
    int32_t v[8];
    for (int r = 0; r < 8; r++) v[r] = (int32_t)in[r * 8 + c] * (int32_t)q[r * 8 + c];
    int32_t o[8];
    IDCT_1D(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o[0], o[1], o[2], o[3], o[4], o[5],
            o[6], o[7]);
    for (int r = 0; r < 8; r++) ws[r * 8 + c] = sat16(DESCALE(o[r], CONST_BITS - PASS1_BITS));
  }
  for (int r = 0; r < 8; r++) {
    const int32_t *w = ws + r * 8;
    int32_t o[8];
    IDCT_1D(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o[0], o[1], o[2], o[3], o[4], o[5],
            o[6], o[7]);
    for (int c = 0; c < 8; c++) out[r * stride + c] = clamp_out(DESCALE(o[c], CONST_BITS + PASS1_BITS + 3));
  }
}

/* zune-jpeg idct_int (stb_image lineage): dequantise, columns then rows */
static void idct_zune(const int16_t *in, const uint16_t *q, uint8_t *out, int stride) {
  int32_t v[64], ws[64];
  for (int i = 0; i < 64; i++) v[i] = (int32_t)in[i] * (int32_t)q[i];
  for (int pass = 0; pass < 2; pass++) {
    const int32_t *s = pass ? ws : v;
    for (int u = 0; u < 8; u++) {
      /* pass 0: column u (stride 8); pass 1: row u (stride 1) */
      const int o = pass ? u * 8 : u, st = pass ? 1 : 8;
      int32_t p2 = s[o + 2 * st], p3 = s[o + 6 * st];
      int32_t p1 = (p2 + p3) * 2217;
      int32_t t2 = p1 + p3 * -7567, t3 = p1 + p2 * 3135;
      p2 = s[o]; p3 = s[o + 4 * st];
      int32_t t0 = (int32_t)((uint32_t)(p2 + p3) << 12), t1 = (int32_t)((uint32_t)(p2 - p3) << 12);
      int32_t x0 = t0 + t3, x3 = t0 - t3, x1 = t1 + t2, x2 = t1 - t2;
      t0 = s[o + 7 * st]; t1 = s[o + 5 * st]; t2 = s[o + 3 * st]; t3 = s[o + st];
      p3 = t0 + t2; int32_t p4 = t1 + t3; p1 = t0 + t3; p2 = t1 + t2;
      int32_t p5 = (p3 + p4) * 4816;
      t0 *= 1223; t1 *= 8410; t2 *= 12586; t3 *= 6149;
      p1 = p5 + p1 * -3685; p2 = p5 + p2 * -10497; p3 = p3 * -8034; p4 = p4 * -1597;
      t3 += p1 + p4; t2 += p2 + p3; t1 += p2 + p4; t0 += p1 + p3;
      const int32_t bias = pass ? 65536 + (128 << 17) : 512, sh = pass ? 17 : 10;
      x0 += bias; x1 += bias; x2 += bias; x3 += bias;
      const int32_t r[8] = {(x0 + t3) >> sh, (x1 + t2) >> sh, (x2 + t1) >> sh, (x3 + t0) >> sh,
                            (x3 - t0) >> sh, (x2 - t1) >> sh, (x1 - t2) >> sh, (x0 - t3) >> sh};
      for (int k = 0; k < 8; k++) {
        if (pass) {
          const int32_t y = r[k];
          out[u * stride + k] = (uint8_t)(y < 0 ? 0 : y > 255 ? 255 : y);
        } else {
          ws[k * 8 + u] = sat16(r[k]);
        }
      }
    }
  }
}

/* zune-jpeg upsample_horizontal over a whole padded row of n >= 2 samples */
static void zune_up_h(const int32_t *in, int n, int32_t *out) {
  out[0] = in[0];
  out[1] = (in[0] * 3 + in[1] + 2) >> 2;
  for (int i = 1; i + 1 < n; i++) {
    const int32_t s = 3 * in[i] + 2;
    out[2 * i] = (s + in[i - 1]) >> 2;
    out[2 * i + 1] = (s + in[i + 1]) >> 2;
  }
  out[2 * n - 2] = (3 * in[n - 2] + in[n - 1] + 2) >> 2;
  out[2 * n - 1] = in[n - 1];
}

/* Upsample component k to full resolution row y, columns [0, W), zune-jpeg style */
static void upsample_row_zune(const oj_jpeg *j, const oj_comp *k, int y, uint8_t *dst) {
  const int hr = j->hmax / k->h, vr = j->vmax / k->v;
  const int pw = k->bw * 8, ph = k->bh * 8;
  const uint8_t *pl = k->plane;
  if (hr == 1 && vr == 1) {
    memcpy(dst, pl + (size_t)y * pw, (size_t)j->W);
    return;
  }
  if (pw < 2) return; /* padded rows are >= 8 samples */
  int32_t *row = (int32_t *)malloc(sizeof(int32_t) * (size_t)pw * 3);
  int32_t *up = row + pw;
  if (vr == 1) {
    for (int x = 0; x < pw; x++) row[x] = pl[(size_t)y * pw + x];
  } else { /* h2v2: vertical first */
    const int r = y >> 1;
    const int rn = (y & 1) ? (r + 1 < ph ? r + 1 : r) : (r > 0 ? r - 1 : 0);
    for (int x = 0; x < pw; x++)
      row[x] = (3 * pl[(size_t)r * pw + x] + 2 + pl[(size_t)rn * pw + x]) >> 2;
  }
  if (pw >= 2) {
    zune_up_h(row, pw, up);
  } else {
    up[0] = up[1] = row[0];
  }
  for (int x = 0; x < j->W; x++) dst[x] = (uint8_t)up[x];
  free(row);
}

static inline uint8_t clamp_i(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* -------------------------------------------------- upsample + colour */

static int32_t Crr[256], Cbb[256], Crg[256], Cbg[256];
static int tables_ready = 0;

static void build_color_tables(void) {
  /* libjpeg jdcolor.c build_ycc_rgb_table, SCALEBITS = 16 */
  const int32_t ONE_HALF = 1 << 15;
  const int32_t F1_40200 = (int32_t)(1.40200 * 65536 + 0.5);
  const int32_t F1_77200 = (int32_t)(1.77200 * 65536 + 0.5);
  const int32_t F0_71414 = (int32_t)(0.71414 * 65536 + 0.5);
  const int32_t F0_34414 = (int32_t)(0.34414 * 65536 + 0.5);
  for (int i = 0; i < 256; i++) {
    int32_t x = i - 128;
    Crr[i] = (F1_40200 * x + ONE_HALF) >> 16;
    Cbb[i] = (F1_77200 * x + ONE_HALF) >> 16;
    Crg[i] = -F0_71414 * x;
    Cbg[i] = -F0_34414 * x + ONE_HALF;
  }
  tables_ready = 1;
}

static inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* Upsample component k of j to full resolution row y, columns [0, W). */
static void upsample_row(const oj_jpeg *j, const oj_comp *k, int y, uint8_t *dst) {
  int hr = j->hmax / k->h, vr = j->vmax / k->v;
  int stride = k->bw * 8;
  const uint8_t *pl = k->plane;
  if (hr == 1 && vr == 1) {
    memcpy(dst, pl + (size_t)y * stride, (size_t)j->W);
    return;
  }
  int fancy = k->dsw > 2;
  if (hr == 2 && vr == 1) {
    const uint8_t *in = pl + (size_t)y * stride;
    for (int x = 0; x < j->W; x++) {
      int c = x >> 1;
      if (!fancy) { dst[x] = in[c]; continue; }
      int a = in[c] * 3;
      if (x & 1) {
        int nb = in[c + 1 < k->dsw ? c + 1 : k->dsw - 1];
        dst[x] = (uint8_t)((a + nb + 2) >> 2);
      } else {
        int nb = in[c > 0 ? c - 1 : 0];
        dst[x] = (uint8_t)((a + nb + 1) >> 2);
      }
    }
    return;
  }
  if (hr == 2 && vr == 2) {
    int r = y >> 1;
    if (!fancy) {
      const uint8_t *in = pl + (size_t)r * stride;
      for (int x = 0; x < j->W; x++) dst[x] = in[x >> 1];
      return;
    }
    int rn = (y & 1) ? r + 1 : r - 1;
    if (rn < 0) rn = 0;
    if (rn > k->dsh - 1) rn = k->dsh - 1;
    const uint8_t *i0 = pl + (size_t)r * stride, *i1 = pl + (size_t)rn * stride;
    for (int x = 0; x < j->W; x++) {
      int c = x >> 1;
      int cs = i0[c] * 3 + i1[c];
      if (x & 1) {
        int cn = c + 1 < k->dsw ? c + 1 : k->dsw - 1;
        int ns = i0[cn] * 3 + i1[cn];
        dst[x] = (uint8_t)((cs * 3 + ns + 7) >> 4);
      } else {
        int cp = c > 0 ? c - 1 : 0;
        int ps = i0[cp] * 3 + i1[cp];
        dst[x] = (uint8_t)((cs * 3 + ps + 8) >> 4);
      }
    }
    return;
  }
}

/* ------------------------------------------------------------- public API */

static int supported_sampling(const oj_jpeg *j) {
  if (j->ncomp == 1) return 1;
  for (int c = 0; c < j->ncomp; c++) {
    if (j->hmax % j->comp[c].h || j->vmax % j->comp[c].v) return 0;
    int hr = j->hmax / j->comp[c].h, vr = j->vmax / j->comp[c].v;
    if (!((hr == 1 && vr == 1) || (hr == 2 && vr == 1) || (hr == 2 && vr == 2))) return 0;
  }
  return 1;
}

/* Header-only probe. */
int oj_info(const uint8_t *d, size_t n, int *w, int *h, int *nc) {
  oj_jpeg j;
  int st = parse_headers(&j, d, n);
  if (st) return st;
  *w = j.W;
  *h = j.H;
  *nc = j.ncomp;
  return OJ_OK;
}

static int decode_to_coefs(oj_jpeg *j, const uint8_t *d, size_t n) {
  int st = parse_headers(j, d, n);
  if (st) return st;
  setup_geometry(j);
  if (!supported_sampling(j)) { free_jpeg(j); return OJ_UNSUPPORTED; }
  for (int c = 0; c < j->ncomp; c++) {
    if (!j->comp[c].coef || !j->comp[c].plane) { free_jpeg(j); return OJ_SMALLBUF; }
    if (!j->qpresent[j->comp[c].tq] ||
        (!j->progressive && (!j->dc[j->comp[c].td].present || !j->ac[j->comp[c].ta].present))) {
      free_jpeg(j);
      return OJ_CORRUPT;
    }
  }
  st = j->progressive ? decode_progressive(j, d, n) : decode_scan(j, d, n);
  if (st) { free_jpeg(j); return st; }
  return OJ_OK;
}

/* Quantized coefficients in decode (MCU-interleaved) order, 64 int16 per block
 * in natural order — the layout the GPU entropy decoder writes. */
int oj_decode_coefs(const uint8_t *d, size_t n, int16_t *out, size_t out_blocks, size_t *nblocks) {
  oj_jpeg j;
  int st = decode_to_coefs(&j, d, n);
  if (st) return st;
  size_t nb = 0;
  if (j.ncomp == 1) {
    oj_comp *k = &j.comp[0];
    int bx_n = (k->dsw + 7) / 8, by_n = (k->dsh + 7) / 8;
    for (int by = 0; by < by_n; by++)
      for (int bx = 0; bx < bx_n; bx++, nb++)
        if (nb < out_blocks) memcpy(out + nb * 64, k->coef + ((size_t)by * k->bw + bx) * 64, 128);
  } else {
    for (int my = 0; my < j.mcuy; my++)
      for (int mx = 0; mx < j.mcux; mx++)
        for (int i = 0; i < (j.progressive ? j.ncomp : j.scan_ncomp); i++) {
          oj_comp *k = &j.comp[j.progressive ? i : j.scan_comp[i]];
          for (int v = 0; v < k->v; v++)
            for (int h = 0; h < k->h; h++, nb++) {
              int by = my * k->v + v, bx = mx * k->h + h;
              if (nb < out_blocks) memcpy(out + nb * 64, k->coef + ((size_t)by * k->bw + bx) * 64, 128);
            }
        }
  }
  *nblocks = nb;
  free_jpeg(&j);
  return nb <= out_blocks ? OJ_OK : OJ_SMALLBUF;
}

/* Full decode to interleaved HWC u8 (1 or 3 channels). */
int oj_decode(const uint8_t *d, size_t n, uint8_t *out, size_t cap, int *w, int *h, int *nc) {
  if (!tables_ready) build_color_tables();
  oj_jpeg j;
  int st = decode_to_coefs(&j, d, n);
  if (st) return st;
  *w = j.W;
  *h = j.H;
  *nc = j.ncomp;
  if ((size_t)j.W * j.H * j.ncomp > cap) { free_jpeg(&j); return OJ_SMALLBUF; }
  for (int c = 0; c < j.ncomp; c++) {
    oj_comp *k = &j.comp[c];
    for (int by = 0; by < k->bh; by++)
      for (int bx = 0; bx < k->bw; bx++)
        (g_sem == OJ_SEM_ZUNE ? idct_zune : idct_islow)(k->coef + ((size_t)by * k->bw + bx) * 64, j.q[k->tq],
                                                         k->plane + (size_t)by * 8 * k->bw * 8 + bx * 8, k->bw * 8);
  }
  if (j.ncomp == 1) {
    for (int y = 0; y < j.H; y++) memcpy(out + (size_t)y * j.W, j.comp[0].plane + (size_t)y * j.comp[0].bw * 8, (size_t)j.W);
    free_jpeg(&j);
    return OJ_OK;
  }
  /* colour space guess: libjpeg jdapimin.c default_decompress_parms */
  int rgb = 0;
  if (j.jfif) rgb = 0;
  else if (j.adobe) rgb = (j.adobe_transform == 0);
  else if (j.comp[0].id == 82 && j.comp[1].id == 71 && j.comp[2].id == 66) rgb = 1;
  uint8_t *r0 = (uint8_t *)malloc((size_t)j.W * 3);
  for (int y = 0; y < j.H; y++) {
    void (*up)(const oj_jpeg *, const oj_comp *, int, uint8_t *) =
        g_sem == OJ_SEM_ZUNE ? upsample_row_zune : upsample_row;
    up(&j, &j.comp[0], y, r0);
    up(&j, &j.comp[1], y, r0 + j.W);
    up(&j, &j.comp[2], y, r0 + 2 * j.W);
    uint8_t *o = out + (size_t)y * j.W * 3;
    for (int x = 0; x < j.W; x++) {
      int Y = r0[x], cb = r0[j.W + x], cr = r0[2 * j.W + x];
      if (rgb) {
        o[3 * x] = (uint8_t)Y; o[3 * x + 1] = (uint8_t)cb; o[3 * x + 2] = (uint8_t)cr;
      } else if (g_sem == OJ_SEM_ZUNE) {
        const int cbp = cb - 128, crp = cr - 128;
        o[3 * x] = clamp_i(Y + ((45 * crp) >> 5));
        o[3 * x + 1] = clamp_i(Y - ((11 * cbp + 23 * crp) >> 5));
        o[3 * x + 2] = clamp_i(Y + ((113 * cbp) >> 6));
      } else {
        o[3 * x] = clamp255(Y + Crr[cr]);
        o[3 * x + 1] = clamp255(Y + ((Cbg[cb] + Crg[cr]) >> 16));
        o[3 * x + 2] = clamp255(Y + Cbb[cb]);
      }
    }
  }
  free(r0);
  free_jpeg(&j);
  return OJ_OK;
}
