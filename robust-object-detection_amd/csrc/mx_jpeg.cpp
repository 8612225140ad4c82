// mx_jpeg.cpp — host half of the hybrid baseline-JPEG decoder: marker parsing and Huffman entropy
// decoding into quantised DCT coefficients (the bitstream of a JPEG without restart markers is one
// sequential prefix-code stream). The device half (mx_jpeg.hip) dequantises, runs the islow IDCT,
// upsamples and converts colour.
//
// Replaces the libjpeg(-turbo) decode behind PIL Image.open(...).convert("RGB")
// (coco_detection_dataset.py:23) and cv2.imread (restore_testsets.py:99, build_corrupted_testsets.py:139).
// Follows ITU-T T.81 (baseline sequential, Huffman): Annex B (markers), F.2.2 (DC/AC decoding,
// EXTEND), C (canonical Huffman tables), and libjpeg's MCU geometry (jdinput.c initial_setup,
// per_scan_setup) for the coefficient layout.
#include <string.h>

#include "../../include/mx_det.h"

namespace mx {
void set_error(const char* fmt, ...);
}

namespace {

// zig-zag index -> natural (row-major) index (T.81 Figure A.6 / libjpeg jpeg_natural_order)
const int kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                          41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                          30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int fail(int code, const char* msg) {
  mx::set_error("%s", msg);
  return code;
}

int cdiv(int a, int b) { return (a + b - 1) / b; }

// Canonical decoding tables (T.81 F.2.2.3: MAXCODE / VALPTR / MINCODE) + a 9-bit lookahead
struct Huff {
  int32_t maxcode[18];
  int32_t valoff[17];
  uint8_t val[256];
  uint8_t look_len[512], look_val[512];  // 0 length: code longer than 9 bits
};

bool huff_counts_ok(const uint8_t* bits);

bool build_huff(const uint8_t* bits, const uint8_t* vals, Huff* h) {
  if (!huff_counts_ok(bits)) return false;
  int code = 0, k = 0;
  int total = 0;
  for (int l = 1; l <= 16; ++l) total += bits[l];
  if (total > 256) return false;
  memcpy(h->val, vals, total);
  memset(h->look_len, 0, sizeof(h->look_len));
  for (int l = 1; l <= 16; ++l) {
    // over-subscription check BEFORE any table write: every code of this length must fit in l bits
    if (code + bits[l] > (1 << l)) return false;
    h->valoff[l] = k - code;  // value index = code + valoff[l]
    for (int i = 0; i < bits[l]; ++i, ++k, ++code) {
      if (l <= 9) {
        const int shift = 9 - l;
        for (int e = 0; e < (1 << shift); ++e) {
          h->look_len[(code << shift) | e] = (uint8_t)l;
          h->look_val[(code << shift) | e] = vals[k];
        }
      }
    }
    h->maxcode[l] = bits[l] ? code - 1 : -1;
    code <<= 1;
  }
  h->maxcode[17] = 0x7fffffff;
  return true;
}

// T.81 C.2 code assignment, checked as libjpeg's jpeg_make_d_derived_tbl does when a scan USES the
// table: after the codes of length l (l up to the longest length in use) the next code must still fit
// in l bits -- no code may be all ones, so a complete table (e.g. two 1-bit codes) is rejected too
// (JERR_BAD_HUFF_TABLE). Tables a scan never uses are not checked (libjpeg derives only used ones).
bool huff_counts_ok(const uint8_t* bits) {
  int last = 0;
  for (int l = 1; l <= 16; ++l)
    if (bits[l]) last = l;
  int code = 0;
  for (int l = 1; l <= last; ++l) {
    code += bits[l];
    if (code >= (1 << l)) return false;
    code <<= 1;
  }
  return true;
}

// JPEG_MAX pixel count accepted on the hybrid path (larger frames decode on the host)
constexpr int64_t kMaxPixels = (int64_t)1 << 28;

struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int cnt = 0;        // valid bits in buf (MSB aligned at bit 63)
  bool marker = false;  // hit a marker: feed zeros (libjpeg does the same)
  void fill() {
    while (cnt <= 56) {
      uint32_t b = 0;
      if (!marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          uint8_t nx = (p + 1 < end) ? p[1] : 0;
          if (nx == 0x00) {
            p += 2;
          } else {  // RSTn / EOI / other marker: stop consuming
            marker = true;
            b = 0;
          }
        } else {
          ++p;
        }
      }
      buf |= (uint64_t)b << (56 - cnt);
      cnt += 8;
    }
  }
  int peek(int n) {
    if (cnt < n) fill();
    return (int)(buf >> (64 - n));
  }
  void skip(int n) {
    buf <<= n;
    cnt -= n;
  }
  int get(int n) {
    if (n == 0) return 0;
    int v = peek(n);
    skip(n);
    return v;
  }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

inline int decode(Bits& b, const Huff& h) {
  const int look = b.peek(9);
  const int l = h.look_len[look];
  if (l) {
    b.skip(l);
    return h.look_val[look];
  }
  int code = b.get(9);
  int len = 9;
  while (len < 17 && code > h.maxcode[len]) {
    code = (code << 1) | b.get(1);
    ++len;
  }
  if (len > 16) return -1;
  return h.val[code + h.valoff[len]];
}

}  // namespace

extern "C" int mx_jpeg_parse(const uint8_t* d, int64_t n, mx_jpeg_info* info) {
  if (!d || !info || n < 4) return fail(MX_EINVAL, "jpeg: null or short buffer");
  memset(info, 0, sizeof(*info));
  if (d[0] != 0xFF || d[1] != 0xD8) return fail(MX_EINVAL, "jpeg: no SOI marker");
  int64_t i = 2;
  bool sof = false, jfif = false, adobe = false;
  int adobe_transform = -1;
  bool qdef[4] = {false, false, false, false};
  while (i + 4 <= n) {
    if (d[i] != 0xFF) {  // extraneous bytes before a marker: skipped, as libjpeg's next_marker does
      ++i;
      continue;
    }
    int m = d[i + 1];
    if (m == 0xFF) { ++i; continue; }  // fill byte
    i += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) break;
    const int len = (d[i] << 8) | d[i + 1];
    if (len < 2 || i + len > n) return fail(MX_EINVAL, "jpeg: truncated segment");
    const uint8_t* s = d + i + 2;
    const int sl = len - 2;
    if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential, Huffman
      if (sl < 6 || s[0] != 8) return fail(MX_EUNSUPPORTED, "jpeg: only 8-bit sequential frames are supported");
      info->height = (s[1] << 8) | s[2];
      info->width = (s[3] << 8) | s[4];
      info->ncomp = s[5];
      if (info->height == 0 || info->width == 0) return fail(MX_EUNSUPPORTED, "jpeg: DNL-defined height");
      if (info->ncomp != 1 && info->ncomp != 3) return fail(MX_EUNSUPPORTED, "jpeg: 1 or 3 components only");
      if ((int64_t)info->height * info->width > kMaxPixels)
        return fail(MX_EUNSUPPORTED, "jpeg: frame larger than 2^28 pixels (decoded on the host)");
      if (sl < 6 + 3 * info->ncomp) return fail(MX_EINVAL, "jpeg: short SOF");
      for (int c = 0; c < info->ncomp; ++c) {
        info->cid[c] = s[6 + 3 * c];
        info->h[c] = s[7 + 3 * c] >> 4;
        info->v[c] = s[7 + 3 * c] & 15;
        info->tq[c] = s[8 + 3 * c];
        if (info->h[c] < 1 || info->h[c] > 2 || info->v[c] < 1 || info->v[c] > 2 || info->tq[c] > 3)
          return fail(MX_EUNSUPPORTED, "jpeg: sampling factors 1..2 and quant tables 0..3 only");
      }
      sof = true;
    } else if ((m >= 0xC2 && m <= 0xC3) || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) ||
               (m >= 0xCD && m <= 0xCF)) {
      return fail(MX_EUNSUPPORTED, "jpeg: progressive / lossless / arithmetic-coded frames are not supported");
    } else if (m == 0xC4) {  // DHT
      int o = 0;
      while (o < sl) {
        const int tc = s[o] >> 4, th = s[o] & 15;
        if (tc > 1 || th > 3 || o + 17 > sl) return fail(MX_EINVAL, "jpeg: bad DHT");
        const int t = tc * 4 + th;
        int tot = 0;
        info->hbits[t][0] = 0;
        for (int l = 1; l <= 16; ++l) {
          info->hbits[t][l] = s[o + l];
          tot += s[o + l];
        }
        if (tot > 256 || o + 17 + tot > sl)
          return fail(MX_EINVAL, "jpeg: bad DHT counts");
        memcpy(info->hval[t], s + o + 17, tot);
        info->hdef[t] = 1;
        o += 17 + tot;
      }
    } else if (m == 0xDB) {  // DQT
      int o = 0;
      while (o < sl) {
        const int pq = s[o] >> 4, tq = s[o] & 15;
        if (tq > 3 || pq > 1 || o + 1 + 64 * (pq + 1) > sl) return fail(MX_EINVAL, "jpeg: bad DQT");
        for (int k = 0; k < 64; ++k)
          info->qt[tq][kNatural[k]] = pq ? (uint16_t)((s[o + 1 + 2 * k] << 8) | s[o + 2 + 2 * k]) : s[o + 1 + k];
        qdef[tq] = true;
        o += 1 + 64 * (pq + 1);
      }
    } else if (m == 0xE0) {  // APP0: a JFIF marker implies YCbCr (jdmarker.c examine_app0)
      if (sl >= 5 && memcmp(s, "JFIF\0", 5) == 0) jfif = true;
    } else if (m == 0xEE) {  // APP14: Adobe colour transform flag (jdmarker.c examine_app14)
      if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) {
        adobe = true;
        adobe_transform = s[11];
      }
    } else if (m == 0xDD) {  // DRI
      if (sl < 2) return fail(MX_EINVAL, "jpeg: bad DRI");
      info->restart_interval = (s[0] << 8) | s[1];
    } else if (m == 0xDA) {  // SOS: the (single, interleaved) scan starts after this header
      if (!sof) return fail(MX_EINVAL, "jpeg: SOS before SOF");
      if (sl < 1) return fail(MX_EINVAL, "jpeg: short SOS");
      const int ns = s[0];
      if (ns != info->ncomp || sl < 1 + 2 * ns + 3)
        return fail(MX_EUNSUPPORTED, "jpeg: only single-scan (all components interleaved) images are supported");
      for (int k = 0; k < ns; ++k) {
        int c = 0;
        while (c < info->ncomp && info->cid[c] != s[1 + 2 * k]) ++c;
        if (c == info->ncomp || c != k) return fail(MX_EUNSUPPORTED, "jpeg: scan component order");
        info->td[c] = s[2 + 2 * k] >> 4;
        info->ta[c] = s[2 + 2 * k] & 15;
        if (info->td[c] > 3 || info->ta[c] > 3 || !info->hdef[info->td[c]] || !info->hdef[4 + info->ta[c]])
          return fail(MX_EINVAL, "jpeg: scan references an undefined Huffman table");
      }
      for (int c = 0; c < info->ncomp; ++c)
        if (!qdef[info->tq[c]]) return fail(MX_EINVAL, "jpeg: component references an undefined quantisation table");
      if (info->ncomp == 3) {
        // libjpeg default_decompress_parms: the colour space of a 3-component frame is YCbCr unless an
        // Adobe marker says transform 0 or (no JFIF / Adobe marker) the component IDs are 'R','G','B';
        // RGB-coded frames have no colour transform and are decoded on the host
        bool rgb = false;
        if (!jfif && adobe) {
          rgb = adobe_transform == 0;
        } else if (!jfif && !adobe) {
          rgb = info->cid[0] == 82 && info->cid[1] == 71 && info->cid[2] == 66;
        }
        if (rgb) return fail(MX_EUNSUPPORTED, "jpeg: RGB-coded frame (no YCbCr transform)");
      }
      const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahl = s[3 + 2 * ns];
      if (ss != 0 || se != 63 || ahl != 0) return fail(MX_EUNSUPPORTED, "jpeg: not a sequential scan");
      info->scan_off = (int32_t)(i + len);
      // geometry (jdinput.c initial_setup / per_scan_setup)
      int hm = 1, vm = 1;
      for (int c = 0; c < info->ncomp; ++c) {
        hm = info->h[c] > hm ? info->h[c] : hm;
        vm = info->v[c] > vm ? info->v[c] : vm;
      }
      if (info->ncomp == 1) {
        info->h[0] = info->v[0] = 1;
        hm = vm = 1;
      }
      info->hmax = hm;
      info->vmax = vm;
      info->mcux = cdiv(info->width, 8 * hm);
      info->mcuy = cdiv(info->height, 8 * vm);
      int64_t off = 0;
      for (int c = 0; c < info->ncomp; ++c) {
        info->bw[c] = info->mcux * info->h[c];
        info->bh[c] = info->mcuy * info->v[c];
        info->dw[c] = cdiv(info->width * info->h[c], hm);
        info->dh[c] = cdiv(info->height * info->v[c], vm);
        info->coef_off[c] = off;
        off += (int64_t)info->bw[c] * info->bh[c] * 64;
      }
      info->coef_total = off;
      if (info->ncomp == 3) {
        const bool ok = info->h[1] == 1 && info->v[1] == 1 && info->h[2] == 1 && info->v[2] == 1 &&
                        !(info->h[0] == 1 && info->v[0] == 2);
        if (!ok) return fail(MX_EUNSUPPORTED, "jpeg: chroma subsampling 4:4:4, 4:2:2 or 4:2:0 only");
      }
      return MX_OK;
    }
    i += len;
  }
  return fail(MX_EINVAL, "jpeg: no scan found");
}

extern "C" int mx_jpeg_decode_coefs(const uint8_t* d, int64_t n, const mx_jpeg_info* info, int16_t* coefs) {
  if (!d || !info || !coefs || info->scan_off <= 0 || info->scan_off > n) return fail(MX_EINVAL, "jpeg: bad arguments");
  Huff dc[4], ac[4];
  for (int c = 0; c < info->ncomp; ++c) {
    if (!build_huff(info->hbits[info->td[c]], info->hval[info->td[c]], &dc[info->td[c]]) ||
        !build_huff(info->hbits[4 + info->ta[c]], info->hval[4 + info->ta[c]], &ac[info->ta[c]]))
      return fail(MX_EINVAL, "jpeg: bad Huffman table");
  }
  memset(coefs, 0, sizeof(int16_t) * (size_t)info->coef_total);
  Bits b;
  b.p = d + info->scan_off;
  b.end = d + n;
  int pred[3] = {0, 0, 0};
  const int64_t nmcu = (int64_t)info->mcux * info->mcuy;
  const int ri = info->restart_interval;
  int64_t left = ri;
  for (int64_t mcu = 0; mcu < nmcu; ++mcu) {
    if (ri && left == 0) {  // restart: byte-align, consume RSTn, reset the DC predictors
      b.buf = 0;
      b.cnt = 0;
      b.marker = false;
      while (b.p + 1 < b.end && !(b.p[0] == 0xFF && b.p[1] >= 0xD0 && b.p[1] <= 0xD7)) ++b.p;
      if (b.p + 1 < b.end) b.p += 2;
      pred[0] = pred[1] = pred[2] = 0;
      left = ri;
    }
    const int64_t my = mcu / info->mcux, mx_ = mcu % info->mcux;
    for (int c = 0; c < info->ncomp; ++c) {
      const Huff& hd = dc[info->td[c]];
      const Huff& ha = ac[info->ta[c]];
      for (int vv = 0; vv < info->v[c]; ++vv)
        for (int hh = 0; hh < info->h[c]; ++hh) {
          const int64_t by = my * info->v[c] + vv, bx = mx_ * info->h[c] + hh;
          int16_t* blk = coefs + info->coef_off[c] + (by * info->bw[c] + bx) * 64;
          int s = decode(b, hd);
          if (s < 0 || s > 11) return fail(MX_EINVAL, "jpeg: corrupt DC code");
          if (s) pred[c] += extend(b.get(s), s);
          blk[0] = (int16_t)pred[c];
          for (int k = 1; k < 64;) {
            const int rs = decode(b, ha);
            if (rs < 0) return fail(MX_EINVAL, "jpeg: corrupt AC code");
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
              k += r;
              if (k > 63) return fail(MX_EINVAL, "jpeg: AC run past the block");
              blk[kNatural[k]] = (int16_t)extend(b.get(sz), sz);
              ++k;
            } else {
              if (r != 15) break;  // EOB
              k += 16;
            }
          }
        }
    }
    if (ri) --left;
  }
  return MX_OK;
}
