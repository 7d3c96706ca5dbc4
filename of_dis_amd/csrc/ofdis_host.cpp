// ofdis_host.cpp -- host-only parts of the C-ABI: parameter tables and validation (run_dense.cpp),
// .flo / .pfm / PNM file formats, and the deterministic synthetic frame-pair generator.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/ofdis.h"

extern "C" {

int ofdis_abi_version(void) { return OFDIS_ABI_VERSION; }

const char *ofdis_status_string(int status) {
  switch (status) {
    case OFDIS_OK: return "ok";
    case OFDIS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case OFDIS_ERR_UNSUPPORTED: return "unsupported parameter combination";
    case OFDIS_ERR_OUT_OF_MEMORY: return "out of memory";
    case OFDIS_ERR_DEVICE: return "HIP runtime error";
    case OFDIS_ERR_NO_DEVICE: return "no gfx950 device";
    case OFDIS_ERR_IO: return "file I/O error";
    default: return "unknown status";
  }
}

// run_dense.cpp:181-184: floor(log2(2 W / (fratio p))) in float, clamped at 0.
int ofdis_auto_first_scale(int imgwidth, int fratio, int patchsize) {
  const float r = std::log2((2.0f * (float)imgwidth) / ((float)fratio * (float)patchsize));
  const int v = (int)std::floor(r);
  return v > 0 ? v : 0;
}

// run_dense.cpp:226-268
int ofdis_params_oppoint(ofdis_params *p, int oppoint, int width_org, int mode, int noc) {
  if (!p || width_org <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  if (mode != OFDIS_MODE_OF && mode != OFDIS_MODE_DE) return OFDIS_ERR_INVALID_ARGUMENT;
  if (noc != 1 && noc != 3) return OFDIS_ERR_INVALID_ARGUMENT;
  std::memset(p, 0, sizeof(*p));
  p->mode = mode;
  p->noc = noc;
  p->dp_thresh = 0.05f;
  p->dr_thresh = 0.95f;
  p->res_thresh = 0.0f;
  p->usefbcon = 0;
  p->patnorm = 1;
  p->costfct = 0;
  p->tv_alpha = 10.0f;
  p->tv_gamma = 10.0f;
  p->tv_delta = 5.0f;
  p->tv_innerit = 1;
  p->tv_solverit = 3;
  p->tv_sor = 1.6f;
  p->verbosity = 2;
  const int fratio = 5;
  int keep = 2;
  switch (oppoint) {
    case 1: p->p_samp_s = 8; p->patove = 0.3f; keep = 2; p->max_iter = p->min_iter = 16; p->usetvref = 0; break;
    case 3: p->p_samp_s = 12; p->patove = 0.75f; keep = 4; p->max_iter = p->min_iter = 16; p->usetvref = 1; break;
    case 4: p->p_samp_s = 12; p->patove = 0.75f; keep = 5; p->max_iter = p->min_iter = 128; p->usetvref = 1; break;
    case 2:
    default: p->p_samp_s = 8; p->patove = 0.4f; keep = 2; p->max_iter = p->min_iter = 12; p->usetvref = 1; break;
  }
  p->sc_f = ofdis_auto_first_scale(width_org, fratio, p->p_samp_s);
  p->sc_l = p->sc_f - keep > 0 ? p->sc_f - keep : 0;
  return OFDIS_OK;
}

// run_dense.cpp:270-295 (atoi / atof of argv[4..23]).
int ofdis_params_from_strings(ofdis_params *p, int count, const char *const *v, int mode, int noc) {
  if (!p || !v || count < 20) return OFDIS_ERR_INVALID_ARGUMENT;
  std::memset(p, 0, sizeof(*p));
  p->mode = mode;
  p->noc = noc;
  int k = 0;
  p->sc_f = std::atoi(v[k++]);
  p->sc_l = std::atoi(v[k++]);
  p->max_iter = std::atoi(v[k++]);
  p->min_iter = std::atoi(v[k++]);
  p->dp_thresh = (float)std::atof(v[k++]);
  p->dr_thresh = (float)std::atof(v[k++]);
  p->res_thresh = (float)std::atof(v[k++]);
  p->p_samp_s = std::atoi(v[k++]);
  p->patove = (float)std::atof(v[k++]);
  p->usefbcon = std::atoi(v[k++]) != 0;
  p->patnorm = std::atoi(v[k++]);
  p->costfct = std::atoi(v[k++]);
  p->usetvref = std::atoi(v[k++]) != 0;
  p->tv_alpha = (float)std::atof(v[k++]);
  p->tv_gamma = (float)std::atof(v[k++]);
  p->tv_delta = (float)std::atof(v[k++]);
  p->tv_innerit = std::atoi(v[k++]);
  p->tv_solverit = std::atoi(v[k++]);
  p->tv_sor = (float)std::atof(v[k++]);
  p->verbosity = std::atoi(v[k++]);
  return OFDIS_OK;
}

int ofdis_params_validate(const ofdis_params *p, int width, int height, int imgpadding) {
  if (!p) return OFDIS_ERR_INVALID_ARGUMENT;
  if (p->mode != OFDIS_MODE_OF && p->mode != OFDIS_MODE_DE) return OFDIS_ERR_INVALID_ARGUMENT;
  if (p->noc != 1 && p->noc != 3) return OFDIS_ERR_INVALID_ARGUMENT;
  if (p->gradmag && p->noc != 1) return OFDIS_ERR_INVALID_ARGUMENT;  // SELECTCHANNEL 2 is single-channel
  if (p->p_samp_s < 2 || (p->p_samp_s & 1)) return OFDIS_ERR_INVALID_ARGUMENT;
  if ((p->p_samp_s * p->p_samp_s * p->noc) % 4) return OFDIS_ERR_INVALID_ARGUMENT;
  if (p->sc_l < 0 || p->sc_f < p->sc_l || p->sc_f > 16) return OFDIS_ERR_INVALID_ARGUMENT;
  if (p->sc_l > 8) return OFDIS_ERR_UNSUPPORTED;  // exact box-mean pyramid
  if (p->costfct < 0 || p->costfct > 2) return OFDIS_ERR_UNSUPPORTED;  // 10 (NCC) unimplemented upstream
  if (p->max_iter < 0 || p->min_iter < 0 || p->tv_innerit < 0 || p->tv_solverit < 0)
    return OFDIS_ERR_INVALID_ARGUMENT;
  if (!(p->patove >= 0.0f && p->patove < 1.0f)) return OFDIS_ERR_INVALID_ARGUMENT;
  if (width > 0 && height > 0) {
    const int d = 1 << p->sc_f;
    if ((width % d) || (height % d)) return OFDIS_ERR_INVALID_ARGUMENT;
    if ((width >> p->sc_f) < 1 || (height >> p->sc_f) < 1) return OFDIS_ERR_INVALID_ARGUMENT;
  }
  if (imgpadding >= 0 && imgpadding < p->p_samp_s) return OFDIS_ERR_INVALID_ARGUMENT;
  return OFDIS_OK;
}

// ------------------------------------------------------------------------------------ files

int ofdis_write_flo(const char *path, const float *flow, int width, int height, int nc) {
  if (!path || !flow || width <= 0 || height <= 0 || nc <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  FILE *f = std::fopen(path, "wb");
  if (!f) return OFDIS_ERR_IO;
  bool ok = std::fwrite("PIEH", 1, 4, f) == 4;
  ok = ok && std::fwrite(&width, sizeof(int), 1, f) == 1 && std::fwrite(&height, sizeof(int), 1, f) == 1;
  const size_t n = (size_t)width * height * nc;
  ok = ok && std::fwrite(flow, sizeof(float), n, f) == n;
  ok = (std::fclose(f) == 0) && ok;
  return ok ? OFDIS_OK : OFDIS_ERR_IO;
}

int ofdis_write_pfm(const char *path, const float *depth, int width, int height) {
  if (!path || !depth || width <= 0 || height <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  FILE *f = std::fopen(path, "wb");
  if (!f) return OFDIS_ERR_IO;
  bool ok = std::fprintf(f, "Pf\n%d %d\n%f\n", width, height, (double)-1.0f) > 0;
  std::vector<float> row(width);
  for (int y = height - 1; y >= 0 && ok; --y) {
    for (int x = 0; x < width; ++x) row[x] = -depth[(size_t)y * width + x];
    ok = std::fwrite(row.data(), sizeof(float), width, f) == (size_t)width;
  }
  ok = (std::fclose(f) == 0) && ok;
  return ok ? OFDIS_OK : OFDIS_ERR_IO;
}

int ofdis_read_flo(const char *path, float *flow, int *width, int *height, int nc) {
  if (!path || !width || !height || nc <= 0) return OFDIS_ERR_INVALID_ARGUMENT;
  FILE *f = std::fopen(path, "rb");
  if (!f) return OFDIS_ERR_IO;
  float tag = 0;
  int w = 0, h = 0;
  bool ok = std::fread(&tag, sizeof(float), 1, f) == 1 && std::fread(&w, sizeof(int), 1, f) == 1 &&
            std::fread(&h, sizeof(int), 1, f) == 1;
  ok = ok && w > 0 && h > 0;
  if (ok && flow) {
    const size_t n = (size_t)w * h * nc;
    ok = std::fread(flow, sizeof(float), n, f) == n;
  }
  std::fclose(f);
  if (!ok) return OFDIS_ERR_IO;
  *width = w;
  *height = h;
  return OFDIS_OK;
}

static int pnm_token(FILE *f) {
  int c = std::fgetc(f);
  while (c == '#' || c == ' ' || c == '\n' || c == '\r' || c == '\t') {
    if (c == '#')
      while (c != '\n' && c != EOF) c = std::fgetc(f);
    c = std::fgetc(f);
  }
  int v = 0;
  if (c < '0' || c > '9') return -1;
  while (c >= '0' && c <= '9') {
    v = v * 10 + (c - '0');
    c = std::fgetc(f);
  }
  return v;
}

int ofdis_read_pnm(const char *path, uint8_t *pixels, int *width, int *height, int *noc, size_t capacity) {
  if (!path || !width || !height || !noc) return OFDIS_ERR_INVALID_ARGUMENT;
  FILE *f = std::fopen(path, "rb");
  if (!f) return OFDIS_ERR_IO;
  char m[2];
  if (std::fread(m, 1, 2, f) != 2 || m[0] != 'P' || (m[1] != '5' && m[1] != '6')) {
    std::fclose(f);
    return OFDIS_ERR_IO;
  }
  const int c = m[1] == '5' ? 1 : 3;
  const int w = pnm_token(f), h = pnm_token(f), maxv = pnm_token(f);
  if (w <= 0 || h <= 0 || maxv != 255) {
    std::fclose(f);
    return OFDIS_ERR_IO;
  }
  *width = w;
  *height = h;
  *noc = c;
  const size_t n = (size_t)w * h * c;
  if (!pixels) {
    std::fclose(f);
    return OFDIS_OK;
  }
  if (capacity < n) {
    std::fclose(f);
    return OFDIS_ERR_INVALID_ARGUMENT;
  }
  const bool ok = std::fread(pixels, 1, n, f) == n;
  std::fclose(f);
  if (!ok) return OFDIS_ERR_IO;
  if (c == 3)  // PPM is RGB; cv::imread returns BGR (run_dense.cpp:205)
    for (size_t i = 0; i < n; i += 3) {
      const uint8_t t = pixels[i];
      pixels[i] = pixels[i + 2];
      pixels[i + 2] = t;
    }
  return OFDIS_OK;
}

// ------------------------------------------------------------------------------------ synthetic pairs

static inline uint64_t splitmix64(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline double gauss(uint64_t &s) {  // Box-Muller
  const double u1 = ((splitmix64(s) >> 11) + 1.0) * (1.0 / 9007199254740994.0);
  const double u2 = (splitmix64(s) >> 11) * (1.0 / 9007199254740992.0);
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

static inline double texture(double x, double y, int c) {
  return 128.0 + 60.0 * std::sin(0.021 * x + 0.3 * std::sin(0.015 * y) + c) * std::cos(0.027 * y) +
         30.0 * std::sin(0.023 * x + 0.017 * y - 0.5 * c);
}

static inline uint8_t to_u8(double v) {
  const long r = std::lround(v);
  return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

// Frame a: band-limited texture + N(0,2) noise.  Frame b samples the same texture at x - u(x,y):
// OF: u = global shift (6.5, 2.25) + rotation <= 0.5 deg + zoom <= 1 % about the centre, varying with
// `frame`; DE: a pure horizontal disparity of -6.5 px.  Noise is independent per frame.
// kind 0: the motion of `mode` above; kind 1: a pure translation by (sx, sy) (the known-answer setups of
// b(x, y) = a(x - sx, y - sy), so the true flow is (sx, sy) everywhere).
static int synth_pair(uint8_t *img_a, uint8_t *img_b, int width, int height, int noc, int frame, int mode,
                      int kind, double sx, double sy) {
  if (!img_a || !img_b || width <= 0 || height <= 0 || (noc != 1 && noc != 3)) return OFDIS_ERR_INVALID_ARGUMENT;
  uint64_t sa = 1234ull + (uint64_t)frame * 2ull, sb = 1235ull + (uint64_t)frame * 2ull;
  const double cx = 0.5 * width, cy = 0.5 * height;
  const double ang = (0.5 * std::sin(0.7 * frame)) * 3.141592653589793 / 180.0;
  const double zoom = 1.0 + 0.01 * std::cos(1.3 * frame);
  const double ca = std::cos(ang) * zoom, sn = std::sin(ang) * zoom;
  const size_t n = (size_t)width * height * noc;
  // the noise streams are sequential (one splitmix64 sequence per frame, pixel-major order) ...
  std::vector<double> na(n), nb(n);
  for (size_t o = 0; o < n; ++o) {
    na[o] = 2.0 * gauss(sa);
    nb[o] = 2.0 * gauss(sb);
  }
  // ... the texture is evaluated row-parallel (same values: every pixel's expression is unchanged)
  auto rows = [&](int y0, int y1) {
    for (int y = y0; y < y1; ++y)
      for (int x = 0; x < width; ++x) {
        double bx, by;
        if (kind == 1) {
          bx = x - sx;
          by = y - sy;
        } else if (mode == OFDIS_MODE_DE) {
          bx = x + 6.5;  // b(x) = a(x + 6.5): disparity -6.5
          by = y;
        } else {
          // inverse of p -> R (p - c) + c + t
          const double qx = x - cx - 6.5, qy = y - cy - 2.25;
          const double det = ca * ca + sn * sn;
          bx = (ca * qx + sn * qy) / det + cx;
          by = (-sn * qx + ca * qy) / det + cy;
        }
        for (int c = 0; c < noc; ++c) {
          const size_t o = ((size_t)y * width + x) * noc + c;
          img_a[o] = to_u8(texture(x, y, c) + na[o]);
          img_b[o] = to_u8(texture(bx, by, c) + nb[o]);
        }
      }
  };
  const int nt = std::max(1, std::min({16, (int)std::thread::hardware_concurrency(), height / 32}));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(rows, (int)((long)height * t / nt), (int)((long)height * (t + 1) / nt));
  rows(0, (int)((long)height / nt));
  for (auto &t : th) t.join();
  return OFDIS_OK;
}

int ofdis_synth_pair_u8(uint8_t *img_a, uint8_t *img_b, int width, int height, int noc, int frame, int mode) {
  return synth_pair(img_a, img_b, width, height, noc, frame, mode, 0, 0.0, 0.0);
}

int ofdis_synth_shift_pair_u8(uint8_t *img_a, uint8_t *img_b, int width, int height, int noc, int frame, float sx,
                              float sy) {
  return synth_pair(img_a, img_b, width, height, noc, frame, OFDIS_MODE_OF, 1, sx, sy);
}

}  // extern "C"
