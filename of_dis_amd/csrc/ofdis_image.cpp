// ofdis_image.cpp -- the on-disk image formats on the input side of the path: what run_dense.cpp's
// cv::imread(path, CV_LOAD_IMAGE_GRAYSCALE / CV_LOAD_IMAGE_COLOR) (run_dense.cpp:202-206) returns, for
// PNG, the Netpbm family and BMP, without OpenCV or libpng (neither is in the image; zlib is).
//
// Restated semantics (OpenCV 3.x/4.x grfmt_png.cpp / grfmt_pxm.cpp over libpng 1.6; both absent here, so
// parity with them is unpinned and pinned instead by tests/test_image_io.py's independent decodes):
//   PNG  every colour type (gray, RGB, palette, gray+alpha, RGBA), bit depths 1/2/4/8/16, Adam7.  The
//        transforms OpenCV asks libpng for, in libpng's order: palette -> RGB, gray 1/2/4 -> 8 bit
//        (x255 / x85 / x17), alpha stripped (not composited), then RGB -> gray (png_set_rgb_to_gray with
//        0.299 / 0.587 -> 15-bit coefficients 9797 / 19234 / 3737: truncating for 8 bit, rounded for 16
//        bit, through libpng's 8-bit gamma tables when a gAMA / sRGB chunk makes the file gamma
//        significant), or gray -> RGB by replication; 16 bit -> 8 bit keeps the high byte
//        (png_set_strip_16); colour output is BGR (png_set_bgr).  CRCs of critical chunks are checked.
//   PNM  P1-P6 (ASCII and binary bitmaps / graymaps / pixmaps), maxval <= 255 taken as is, 65535 -> high
//        byte; colour -> gray by OpenCV's fixed-point icvCvt_BGR2Gray_8u_C3C1R
//        ((1868 B + 9617 G + 4899 R + 8192) >> 14); colour output is BGR.
//   BMP  OpenCV's BmpDecoder (grfmt_bmp.cpp): see decode_bmp.
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/ofdis.h"

namespace {

struct Image {
  int w = 0, h = 0, c = 0;  // c = 1 or 3 (BGR), 8 bit
  std::vector<uint8_t> px;
};

bool read_file(const char *path, std::vector<uint8_t> &buf) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  uint8_t tmp[1 << 16];
  size_t k;
  while ((k = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + k);
  const bool ok = !std::ferror(f);
  std::fclose(f);
  return ok;
}

// ------------------------------------------------------------------------------------------- PNG

inline uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// png_gamma_8bit_correct (libpng png.c): floor(255 * (v/255)^(g/1e5) + .5) for 0 < v < 255.
uint8_t gamma8(unsigned v, double g) {
  if (v == 0 || v >= 255) return (uint8_t)v;
  return (uint8_t)std::floor(255.0 * std::pow(v / 255.0, g * 0.00001) + 0.5);
}
// png_reciprocal: floor(1e10 / a + .5)
long reciprocal(long a) { return (long)std::floor(1e10 / (double)a + 0.5); }
bool gamma_significant(long g) { return g < 100000 - 5000 || g > 100000 + 5000; }

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Reverse the per-row filters of one (sub-)image in place; rows of `rb` bytes, `bpp` bytes per pixel
// (at least 1).  Returns false on an unknown filter type.
bool unfilter(uint8_t *data, int rows, size_t rb, int bpp) {
  std::vector<uint8_t> prev(rb, 0);
  uint8_t *out = data;  // rows are compacted in place: out lags the input by one byte per row
  const uint8_t *in = data;
  const size_t bp = (size_t)bpp < rb ? (size_t)bpp : rb;
  for (int y = 0; y < rows; ++y) {
    const int ft = *in++;
    uint8_t *cur = out;
    std::memmove(cur, in, rb);
    in += rb;
    const uint8_t *pv = prev.data();
    // one loop per filter type (the first bpp bytes have no left neighbour: a = c = 0)
    switch (ft) {
      case 0: break;
      case 1:
        for (size_t i = bp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + cur[i - bpp]);
        break;
      case 2:
        for (size_t i = 0; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + pv[i]);
        break;
      case 3:
        for (size_t i = 0; i < bp; ++i) cur[i] = (uint8_t)(cur[i] + (pv[i] >> 1));
        for (size_t i = bp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + ((cur[i - bpp] + pv[i]) >> 1));
        break;
      case 4:
        for (size_t i = 0; i < bp; ++i) cur[i] = (uint8_t)(cur[i] + paeth(0, pv[i], 0));
        for (size_t i = bp; i < rb; ++i) cur[i] = (uint8_t)(cur[i] + paeth(cur[i - bpp], pv[i], pv[i - bpp]));
        break;
      default: return false;
    }
    std::memcpy(prev.data(), cur, rb);
    out += rb;
  }
  return true;
}

// Sample s of row `row` (unpacked, big-endian for 16 bit) -> value in [0, 2^depth).
inline unsigned sample(const uint8_t *row, size_t s, int depth) {
  switch (depth) {
    case 16: return (unsigned)row[2 * s] << 8 | row[2 * s + 1];
    case 8: return row[s];
    default: {
      const size_t bit = s * depth;
      return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1);
    }
  }
}

constexpr uint64_t kMaxImagePixels = 1ull << 30;

int decode_png(const std::vector<uint8_t> &f, int want, Image &img, bool header_only = false) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return OFDIS_ERR_IO;
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte;
  long file_gamma = 0;  // 1e5 units, 0 = none
  bool srgb = false, seen_ihdr = false, seen_iend = false;
  size_t pos = 8;
  while (pos + 12 <= f.size()) {
    const uint32_t len = be32(&f[pos]);
    if (len > f.size() - pos - 12) return OFDIS_ERR_IO;
    const uint8_t *type = &f[pos + 4], *data = &f[pos + 8];
    const bool critical = !(type[0] & 0x20);
    const uint32_t crc = be32(&f[pos + 8 + len]);
    if (critical && (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4) != crc) return OFDIS_ERR_IO;
    if (!std::memcmp(type, "IHDR", 4)) {
      if (len != 13) return OFDIS_ERR_IO;
      W = be32(data);
      H = be32(data + 4);
      depth = data[8];
      ctype = data[9];
      interlace = data[12];
      if (data[10] != 0 || data[11] != 0 || interlace > 1) return OFDIS_ERR_IO;
      seen_ihdr = true;
    } else if (!std::memcmp(type, "PLTE", 4)) {
      plte.assign(data, data + len);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), data, data + len);
    } else if (!std::memcmp(type, "gAMA", 4)) {
      if (len == 4) file_gamma = (long)be32(data);
    } else if (!std::memcmp(type, "sRGB", 4)) {
      srgb = true;
    } else if (!std::memcmp(type, "IEND", 4)) {
      seen_iend = true;
      break;
    }
    pos += 12 + len;
  }
  if (!seen_ihdr || !seen_iend || W == 0 || H == 0 || W > (1u << 24) || H > (1u << 24)) return OFDIS_ERR_IO;
  // OpenCV's CV_IO_MAX_IMAGE_PIXELS (2^30): refuse before sizing any buffer from the header alone
  if ((uint64_t)W * H > kMaxImagePixels) return OFDIS_ERR_IO;
  int nch;
  switch (ctype) {
    case 0: nch = 1; if (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16) return OFDIS_ERR_IO; break;
    case 2: nch = 3; if (depth != 8 && depth != 16) return OFDIS_ERR_IO; break;
    case 3: nch = 1; if (depth != 1 && depth != 2 && depth != 4 && depth != 8) return OFDIS_ERR_IO; break;
    case 4: nch = 2; if (depth != 8 && depth != 16) return OFDIS_ERR_IO; break;
    case 6: nch = 4; if (depth != 8 && depth != 16) return OFDIS_ERR_IO; break;
    default: return OFDIS_ERR_IO;
  }
  if (header_only) {  // a size query (pixels == NULL): the chunk structure, CRCs and header checked, nothing inflated
    img.w = (int)W;
    img.h = (int)H;
    img.c = want;
    return OFDIS_OK;
  }
  if (ctype == 3 && (plte.empty() || plte.size() % 3)) return OFDIS_ERR_IO;
  const int bpp = std::max(1, nch * depth / 8);
  auto row_bytes = [&](uint32_t w) { return ((size_t)w * nch * depth + 7) / 8; };

  // inflate: the exact size of the filtered stream is known
  static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  size_t raw_size = 0;
  if (!interlace) {
    raw_size = (row_bytes(W) + 1) * H;
  } else {
    for (int pss = 0; pss < 7; ++pss) {
      const uint32_t pw = (W + adx[pss] - 1 - ax0[pss]) / adx[pss], ph = (H + ady[pss] - 1 - ay0[pss]) / ady[pss];
      if (pw && ph) raw_size += (row_bytes(pw) + 1) * ph;
    }
  }
  std::vector<uint8_t> raw(raw_size + 1);
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit(&zs) != Z_OK) return OFDIS_ERR_OUT_OF_MEMORY;
  zs.next_in = idat.data();
  zs.avail_in = (uInt)idat.size();
  zs.next_out = raw.data();
  zs.avail_out = (uInt)raw.size();
  const int zr = inflate(&zs, Z_FINISH);
  const size_t got = raw.size() - zs.avail_out;
  inflateEnd(&zs);
  if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR) || got < raw_size) return OFDIS_ERR_IO;

  // unfilter and de-interlace into full-size unpacked rows of samples (16-bit values kept)
  std::vector<uint16_t> smp((size_t)W * H * nch);
  auto put_rows = [&](uint8_t *sub, uint32_t pw, uint32_t ph, int x0, int y0, int dx, int dy) -> bool {
    const size_t rb = row_bytes(pw);
    if (!unfilter(sub, (int)ph, rb, bpp)) return false;
    for (uint32_t y = 0; y < ph; ++y) {
      const uint8_t *r = sub + y * rb;
      uint16_t *dst = &smp[((size_t)(y0 + y * dy) * W) * nch];
      if (depth == 8 && dx == 1 && x0 == 0) {  // the common case: one byte per sample, a whole row
        for (size_t i = 0; i < (size_t)pw * nch; ++i) dst[i] = r[i];
        continue;
      }
      for (uint32_t x = 0; x < pw; ++x)
        for (int k = 0; k < nch; ++k) dst[(size_t)(x0 + x * dx) * nch + k] = (uint16_t)sample(r, (size_t)x * nch + k, depth);
    }
    return true;
  };
  if (!interlace) {
    if (!put_rows(raw.data(), W, H, 0, 0, 1, 1)) return OFDIS_ERR_IO;
  } else {
    uint8_t *p = raw.data();
    for (int pss = 0; pss < 7; ++pss) {
      const uint32_t pw = (W + adx[pss] - 1 - ax0[pss]) / adx[pss], ph = (H + ady[pss] - 1 - ay0[pss]) / ady[pss];
      if (!pw || !ph) continue;
      if (!put_rows(p, pw, ph, ax0[pss], ay0[pss], adx[pss], ady[pss])) return OFDIS_ERR_IO;
      p += (row_bytes(pw) + 1) * ph;
    }
  }

  // libpng's transform chain as OpenCV configures it
  const bool color_src = (ctype & 2) != 0;  // PNG_COLOR_MASK_COLOR (palette included)
  const bool d16 = depth == 16;
  // gamma: png_init_read_transformations -- no gAMA/sRGB: gamma = screen = 1 (tables unused)
  long g = file_gamma > 0 ? file_gamma : (srgb ? 45455 : 0);
  const bool use_gamma = color_src && want == 1 && g > 0 && gamma_significant(g);
  if (use_gamma && d16) return OFDIS_ERR_UNSUPPORTED;  // libpng's 16-bit gamma tables: not restated
  uint8_t to1[256], from1[256];
  if (use_gamma) {
    const long screen = reciprocal(g);  // "assume the output matches the input"
    const long g_to1 = reciprocal(g), g_from1 = reciprocal(screen);
    for (unsigned v = 0; v < 256; ++v) {
      to1[v] = gamma_significant(g_to1) ? gamma8(v, (double)g_to1) : (uint8_t)v;
      from1[v] = gamma_significant(g_from1) ? gamma8(v, (double)g_from1) : (uint8_t)v;
    }
  }
  const uint32_t rc = 9797, gc = 19234, bc = 32768 - rc - gc;  // png_set_rgb_to_gray(png, 1, 0.299, 0.587)
  img.w = (int)W;
  img.h = (int)H;
  img.c = want;
  img.px.assign((size_t)W * H * want, 0);
  for (size_t i = 0; i < (size_t)W * H; ++i) {
    const uint16_t *s = &smp[i * nch];
    unsigned r, gg, b;  // at the stream's depth after expansion (8, or 16 for 16-bit files)
    if (ctype == 3) {
      const unsigned idx = s[0];
      if ((size_t)idx * 3 + 2 >= plte.size()) return OFDIS_ERR_IO;
      r = plte[3 * idx]; gg = plte[3 * idx + 1]; b = plte[3 * idx + 2];
    } else if (color_src) {
      r = s[0]; gg = s[1]; b = s[2];
    } else {
      unsigned v = s[0];
      if (depth < 8) v *= depth == 1 ? 255 : (depth == 2 ? 0x55 : 0x11);  // png_do_expand
      r = gg = b = v;
    }
    if (want == 1) {
      unsigned gray;
      if (!color_src) {
        gray = r;
      } else if (d16) {
        gray = (rc * r + gc * gg + bc * b + 16384) >> 15;  // 16-bit: rounded (libpng >= 1.5.5)
      } else if (r == gg && r == b) {
        gray = r;
      } else if (use_gamma) {
        gray = from1[(rc * to1[r] + gc * to1[gg] + bc * to1[b] + 16384) >> 15];
      } else {
        gray = (rc * r + gc * gg + bc * b) >> 15;  // "the historical approach which simply truncates"
      }
      img.px[i] = (uint8_t)(d16 ? gray >> 8 : gray);  // png_set_strip_16
    } else {
      uint8_t *d = &img.px[i * 3];
      d[0] = (uint8_t)(d16 ? b >> 8 : b);  // png_set_bgr
      d[1] = (uint8_t)(d16 ? gg >> 8 : gg);
      d[2] = (uint8_t)(d16 ? r >> 8 : r);
    }
  }
  return OFDIS_OK;
}

// ------------------------------------------------------------------------------------------- PNM

struct Cursor {
  const std::vector<uint8_t> &f;
  size_t p = 0;
  int token() {  // next decimal integer, skipping whitespace and # comments; -1 on error
    while (p < f.size()) {
      const int c = f[p];
      if (c == '#') {
        while (p < f.size() && f[p] != '\n' && f[p] != '\r') ++p;
      } else if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') {
        ++p;
      } else {
        break;
      }
    }
    if (p >= f.size() || f[p] < '0' || f[p] > '9') return -1;
    long v = 0;
    while (p < f.size() && f[p] >= '0' && f[p] <= '9') {
      v = v * 10 + (f[p++] - '0');
      if (v > (1 << 24)) return -1;
    }
    return (int)v;
  }
};

int decode_pnm(const std::vector<uint8_t> &f, int want, Image &img) {
  if (f.size() < 3 || f[0] != 'P' || f[1] < '1' || f[1] > '6') return OFDIS_ERR_IO;
  const int kind = f[1] - '0';
  const bool ascii = kind <= 3, bitmap = kind == 1 || kind == 4;
  const int nch = (kind == 3 || kind == 6) ? 3 : 1;
  Cursor cur{f, 2};
  const int w = cur.token(), h = cur.token();
  const int maxv = bitmap ? 1 : cur.token();
  if (w <= 0 || h <= 0 || maxv <= 0 || (maxv > 255 && maxv != 65535)) return OFDIS_ERR_IO;
  if ((uint64_t)w * h > kMaxImagePixels) return OFDIS_ERR_IO;
  const size_t n = (size_t)w * h * nch;
  std::vector<unsigned> v(n);
  if (ascii) {
    for (size_t i = 0; i < n; ++i) {
      if (kind == 1) {  // P1 digits may be unseparated
        while (cur.p < f.size() && !(f[cur.p] == '0' || f[cur.p] == '1')) {
          if (f[cur.p] == '#')
            while (cur.p < f.size() && f[cur.p] != '\n') ++cur.p;
          else
            ++cur.p;
        }
        if (cur.p >= f.size()) return OFDIS_ERR_IO;
        v[i] = f[cur.p++] == '1' ? 0 : 255;  // PBM: 1 = black
      } else {
        const int t = cur.token();
        if (t < 0 || t > maxv) return OFDIS_ERR_IO;
        v[i] = maxv == 65535 ? (unsigned)t >> 8 : (unsigned)t;
      }
    }
  } else {
    size_t p = cur.p + 1;  // exactly one whitespace byte after the header
    if (kind == 4) {
      const size_t rb = ((size_t)w + 7) / 8;
      if (p + rb * h > f.size()) return OFDIS_ERR_IO;
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) v[(size_t)y * w + x] = (f[p + y * rb + (x >> 3)] >> (7 - (x & 7))) & 1 ? 0 : 255;
    } else if (maxv == 65535) {
      if (p + 2 * n > f.size()) return OFDIS_ERR_IO;
      for (size_t i = 0; i < n; ++i) v[i] = f[p + 2 * i];  // high byte of the big-endian sample
    } else {
      if (p + n > f.size()) return OFDIS_ERR_IO;
      for (size_t i = 0; i < n; ++i) v[i] = f[p + i];
    }
  }
  img.w = w;
  img.h = h;
  img.c = want;
  img.px.assign((size_t)w * h * want, 0);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    if (nch == 1) {
      for (int k = 0; k < want; ++k) img.px[i * want + k] = (uint8_t)v[i];
    } else if (want == 3) {
      img.px[3 * i] = (uint8_t)v[3 * i + 2];  // RGB file -> BGR
      img.px[3 * i + 1] = (uint8_t)v[3 * i + 1];
      img.px[3 * i + 2] = (uint8_t)v[3 * i];
    } else {  // icvCvt_BGR2Gray_8u_C3C1R, SCALE 14: cB 1868, cG 9617, cR 4899, descale with rounding
      img.px[i] = (uint8_t)((v[3 * i + 2] * 1868u + v[3 * i + 1] * 9617u + v[3 * i] * 4899u + 8192u) >> 14);
    }
  }
  return OFDIS_OK;
}

// ------------------------------------------------------------------------------------------- BMP
// OpenCV's BmpDecoder (grfmt_bmp.cpp), restated: BITMAPINFOHEADER and its V4 / V5 extensions (40 / 108 / 124-byte
// headers) and the OS/2 BITMAPCOREHEADER (12 bytes, 3-byte palette entries); 1 / 4 / 8-bit palette images,
// 16-bit 5-5-5 (BI_RGB, or BI_BITFIELDS with those masks) and 5-6-5 (BI_BITFIELDS), 24-bit BGR and 32-bit BGRX
// (BI_RGB or BI_BITFIELDS with the standard masks: alpha dropped); bottom-up rows unless the height is negative,
// rows padded to 4 bytes.  Colour output is the stored BGR (5-bit fields as (v << 3) & 0xf8 -- no bit
// replication, icvCvt_BGR5552BGR_8u_C2C3R / icvCvt_BGR5652BGR_8u_C2C3R); gray output is the fixed-point
// icvCvt_BGR2Gray_8u ((1868 B + 9617 G + 4899 R + 8192) >> 14) of those values -- of the palette entries for
// palette images (CvtPaletteToGray).  RLE4 / RLE8 and other masks: OFDIS_ERR_UNSUPPORTED.
inline uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }

int decode_bmp(const std::vector<uint8_t> &f, int want, Image &img) {
  if (f.size() < 26 || f[0] != 'B' || f[1] != 'M') return OFDIS_ERR_IO;
  const uint32_t off = le32(&f[10]), hsz = le32(&f[14]);
  int64_t w, h;
  int bpp;
  uint32_t comp = 0, nclr = 0;
  size_t pal_at, pal_entry;
  if (hsz == 12) {  // BITMAPCOREHEADER
    w = le16(&f[18]);
    h = (int16_t)le16(&f[20]);
    bpp = le16(&f[24]);
    pal_at = 14 + 12;
    pal_entry = 3;
  } else if (hsz == 40 || hsz == 52 || hsz == 56 || hsz == 108 || hsz == 124) {
    if (f.size() < 14 + 40) return OFDIS_ERR_IO;
    w = (int32_t)le32(&f[18]);
    h = (int32_t)le32(&f[22]);
    bpp = le16(&f[28]);
    comp = le32(&f[30]);
    nclr = le32(&f[46]);
    pal_at = 14 + hsz;
    pal_entry = 4;
  } else {
    return OFDIS_ERR_UNSUPPORTED;
  }
  const bool top_down = h < 0;
  if (top_down) h = -h;
  if (w <= 0 || h <= 0 || (uint64_t)w * (uint64_t)h > kMaxImagePixels) return OFDIS_ERR_IO;
  // pixel format
  enum { kPal, k555, k565, k24, k32 } fmt;
  if (bpp == 1 || bpp == 4 || bpp == 8) {
    if (comp != 0) return OFDIS_ERR_UNSUPPORTED;  // RLE8 / RLE4
    fmt = kPal;
  } else if (bpp == 16 || bpp == 32) {
    uint32_t rm = bpp == 16 ? 0x7c00 : 0xff0000, gm = bpp == 16 ? 0x03e0 : 0xff00, bm = bpp == 16 ? 0x001f : 0xff;
    if (comp == 3) {  // BI_BITFIELDS: masks after the 40-byte header (or inside a V4 / V5 header)
      if (hsz < 40 || f.size() < 14 + 40 + 12) return OFDIS_ERR_IO;
      rm = le32(&f[54]);
      gm = le32(&f[58]);
      bm = le32(&f[62]);
      if (hsz == 40) pal_at += 12;
    } else if (comp != 0) {
      return OFDIS_ERR_UNSUPPORTED;
    }
    if (bpp == 16 && rm == 0x7c00 && gm == 0x03e0 && bm == 0x001f) fmt = k555;
    else if (bpp == 16 && rm == 0xf800 && gm == 0x07e0 && bm == 0x001f) fmt = k565;
    else if (bpp == 32 && rm == 0xff0000 && gm == 0xff00 && bm == 0xff) fmt = k32;
    else return OFDIS_ERR_UNSUPPORTED;
  } else if (bpp == 24) {
    if (comp != 0) return OFDIS_ERR_UNSUPPORTED;
    fmt = k24;
  } else {
    return OFDIS_ERR_UNSUPPORTED;
  }
  // palette (BGR[X] entries): clrUsed or 2^bpp of them
  uint8_t pal[256][3] = {};
  if (fmt == kPal) {
    const uint32_t n = nclr ? nclr : (1u << bpp);
    if (n > 256 || pal_at + (size_t)n * pal_entry > f.size()) return OFDIS_ERR_IO;
    for (uint32_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) pal[i][k] = f[pal_at + i * pal_entry + k];
  }
  const size_t stride = (((size_t)w * bpp + 31) / 32) * 4;
  if (off >= f.size() || off + stride * (size_t)h > f.size()) return OFDIS_ERR_IO;
  img.w = (int)w;
  img.h = (int)h;
  img.c = want;
  img.px.assign((size_t)w * h * want, 0);
  auto put = [&](size_t i, unsigned b, unsigned g, unsigned r) {
    if (want == 3) {
      img.px[3 * i] = (uint8_t)b;
      img.px[3 * i + 1] = (uint8_t)g;
      img.px[3 * i + 2] = (uint8_t)r;
    } else {
      img.px[i] = (uint8_t)((b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14);
    }
  };
  for (int64_t y = 0; y < h; ++y) {
    const uint8_t *row = &f[off + stride * (size_t)(top_down ? y : h - 1 - y)];
    for (int64_t x = 0; x < w; ++x) {
      const size_t i = (size_t)y * w + x;
      switch (fmt) {
        case kPal: {
          unsigned idx;
          if (bpp == 8) idx = row[x];
          else if (bpp == 4) idx = (row[x >> 1] >> ((x & 1) ? 0 : 4)) & 15;
          else idx = (row[x >> 3] >> (7 - (x & 7))) & 1;
          put(i, pal[idx][0], pal[idx][1], pal[idx][2]);
          break;
        }
        case k555: {
          const unsigned t = le16(row + 2 * x);
          put(i, (t << 3) & 0xf8, (t >> 2) & 0xf8, (t >> 7) & 0xf8);
          break;
        }
        case k565: {
          const unsigned t = le16(row + 2 * x);
          put(i, (t << 3) & 0xf8, (t >> 3) & 0xfc, (t >> 8) & 0xf8);
          break;
        }
        case k24: put(i, row[3 * x], row[3 * x + 1], row[3 * x + 2]); break;
        case k32: put(i, row[4 * x], row[4 * x + 1], row[4 * x + 2]); break;
      }
    }
  }
  return OFDIS_OK;
}

}  // namespace

extern "C" {

int ofdis_read_image(const char *path, uint8_t *pixels, int *width, int *height, int want_noc, size_t capacity) {
  if (!path || !width || !height || (want_noc != 1 && want_noc != 3)) return OFDIS_ERR_INVALID_ARGUMENT;
  try {  // no C++ exception may cross the C-ABI: a failed allocation becomes a status code
    std::vector<uint8_t> f;
    if (!read_file(path, f)) return OFDIS_ERR_IO;
    Image img;
    int rc;
    if (f.size() >= 8 && f[0] == 137 && f[1] == 'P' && f[2] == 'N' && f[3] == 'G')
      rc = decode_png(f, want_noc, img, pixels == nullptr);
    else if (f.size() >= 2 && f[0] == 'P' && f[1] >= '1' && f[1] <= '6')
      rc = decode_pnm(f, want_noc, img);
    else if (f.size() >= 2 && f[0] == 'B' && f[1] == 'M')
      rc = decode_bmp(f, want_noc, img);
    else
      rc = OFDIS_ERR_UNSUPPORTED;
    if (rc) return rc;
    *width = img.w;
    *height = img.h;
    if (!pixels) return OFDIS_OK;
    if (capacity < img.px.size()) return OFDIS_ERR_INVALID_ARGUMENT;
    std::memcpy(pixels, img.px.data(), img.px.size());
    return OFDIS_OK;
  } catch (const std::bad_alloc &) {
    return OFDIS_ERR_OUT_OF_MEMORY;
  } catch (...) {
    return OFDIS_ERR_IO;
  }
}

}  // extern "C"
