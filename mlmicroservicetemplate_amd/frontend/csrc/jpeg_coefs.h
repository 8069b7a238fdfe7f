// Host half of the GPU JPEG path (reference contract: an uploaded image FILE that
// the model decodes, reference src/model/model.py:16-23).  The serial part of baseline JPEG --
// marker parsing and Huffman (entropy) decoding -- runs here on the native front end's I/O threads;
// everything per pixel (IDCT, chroma upsampling, YCbCr -> RGB, the resize + centre crop of the
// PIL reference pipeline, plugins/builtin.py decode_image) runs in ops/csrc/image_decode.hip on the
// GPU as the first kernels of the serving graph.
//
// The unit handed to the GPU is a fixed-size "image container" (engine slot row):
//   [0, 64)   header (ImgHeader)
//   [64, ..)  kind RAW:  224 x 224 x 3 uint8 RGB (an already-decoded / raw upload)
//             kind JPEG (all offsets relative to the payload):
//               [0, 384)        qtab: per component, 64 u16 quantisation steps in natural order
//               [384, ..)       gstart: u32 per group of 64 blocks = entry offset of its first block
//               [counts_off ..) counts: u8 per block = its entry units
//               [entries_off..) entries, 2-byte units in block-table order: (int8 quantised value,
//                               u8 natural position r * s + c in the kept s x s corner); a value
//                               outside int8 is the escape (0x80, pos) followed by one unit holding
//                               the int16 value.
//             Blocks are numbered component-major, each component's MCU-padded grid in raster order.
//             Compact because a 640 x 480 camera JPEG has ~7 k blocks and 40-70 k nonzero
//             coefficients: dense int16 blocks alone would be 0.9 MB.
// s = 8 / d where d is the DCT-domain downscale PIL's draft() would pick for a 256-pixel shorter
// side (d = largest of 8, 4, 2, 1 <= min(W // 256, H // 256)); when the entries still exceed the
// container, d doubles until they fit (flagged: a coarser decode than PIL's).  The resize /
// crop geometry of decode_image (shorter side 256, bilinear, centre 224) is computed here with
// Python's rounding so the device pass reproduces it.
//
// Baseline (SOF0) and extended-sequential Huffman (SOF1, 8-bit) JPEGs, 1 or 3 components,
// any sampling factors up to 2 x 2, restart intervals.  Progressive / arithmetic / 12-bit / CMYK
// streams are refused (the caller falls back to the PIL decode threads).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace mlsjpeg {

constexpr uint32_t IMG_MAGIC = 0x4A534C4Du;  // "MLSJ"
constexpr int IMG_OUT = 224;                 // model input side
constexpr int IMG_SHORT = 256;               // decode_image's `resize`
constexpr int HDR_BYTES = 64;
constexpr size_t PAYLOAD_BYTES = (size_t)IMG_OUT * IMG_OUT * 3;
constexpr size_t CONTAINER_BYTES = HDR_BYTES + PAYLOAD_BYTES;
// device scratch per image (ops/csrc/image_decode.hip): component planes + RGB + the horizontal
// resample pass must fit; decode_at() moves to a coarser DCT scale until they do
constexpr size_t SCRATCH_PER_IMAGE = (size_t)2 << 20;  // fits PIL-drafted sizes (short side 256..511)
enum Kind : uint32_t { KIND_RAW = 0, KIND_JPEG = 1 };

#pragma pack(push, 1)
struct CompHdr {
  uint8_t h, v;      // sampling factors
  uint16_t bw, bh;   // blocks per row / column (MCU grid)
  uint32_t offset;   // index of this component's first block in the block table
};
struct ImgHeader {
  uint32_t magic, kind;
  uint16_t width, height;  // decoded (DCT-scaled) image size
  uint8_t ncomp, s, hmax, vmax;
  CompHdr comp[3];
  uint16_t rw, rh;      // resized size (shorter side IMG_SHORT)
  uint16_t left, top;   // centre crop offset in the resized image
  uint8_t coarser;      // 1: decoded at a smaller scale than PIL's draft (container budget)
  uint32_t nblocks;     // DCT blocks (all components)
  uint32_t entries_off; // payload byte offset of the entry units (counts_off = 384 + 4 * groups)
  uint8_t pad[HDR_BYTES - 4 - 4 - 4 - 4 - 3 * 10 - 8 - 1 - 8];
};
#pragma pack(pop)
static_assert(sizeof(ImgHeader) == HDR_BYTES, "container header");

// false: the resized size does not fit the header's 16-bit fields (aspect ratio beyond ~256:1);
// the caller then takes the PIL path
inline bool fill_geometry(ImgHeader& h) {
  // decode_image: s = resize / min(w, h); nw, nh = max(size, round(w * s)), max(size, round(h * s))
  const double sc = (double)IMG_SHORT / (double)(h.width < h.height ? h.width : h.height);
  const double nw = std::nearbyint(h.width * sc), nh = std::nearbyint(h.height * sc);  // half-to-even
  if (nw > 65535.0 || nh > 65535.0) return false;
  h.rw = (uint16_t)(nw < IMG_OUT ? IMG_OUT : nw);
  h.rh = (uint16_t)(nh < IMG_OUT ? IMG_OUT : nh);
  h.left = (uint16_t)((h.rw - IMG_OUT) / 2);
  h.top = (uint16_t)((h.rh - IMG_OUT) / 2);
  return true;
}

// a raw 224 x 224 x 3 RGB upload -> container
inline void raw_container(const uint8_t* rgb, uint8_t* out) {
  ImgHeader h;
  std::memset(&h, 0, sizeof(h));
  h.magic = IMG_MAGIC;
  h.kind = KIND_RAW;
  h.width = h.height = IMG_OUT;
  h.ncomp = 3;
  h.rw = h.rh = IMG_OUT;
  std::memcpy(out, &h, sizeof(h));
  std::memcpy(out + HDR_BYTES, rgb, PAYLOAD_BYTES);
}

static const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  // canonical code tables: for code length l, codes [mincode[l], maxcode[l]] map to vals[valptr[l] + ...]
  int maxcode[18], valptr[17], mincode[17];
  uint8_t vals[256];
  // fast path: 9-bit lookahead -> (length << 8) | value, 0 = slow path
  uint16_t fast[512];
  // combined path (FAST_BITS lookahead): symbol AND its magnitude bits when code + extra bits fit
  // -- one lookup per coefficient for most codes (the libjpeg-turbo idea, own table layout):
  // bits 0-7 symbol, 8-11 code length, 12-15 total length (0 = not combined), value in `val`
  uint16_t comb[1 << 10];
  int16_t val[1 << 10];
  bool ok = false;
};
constexpr int FAST_BITS = 10;

inline bool build_huff(Huff& t, const uint8_t* counts, const uint8_t* symbols, int nsym) {
  std::memset(t.fast, 0, sizeof(t.fast));
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    t.valptr[l] = k;
    t.mincode[l] = code;
    code += counts[l - 1];
    k += counts[l - 1];
    if (code > (1 << l)) return false;
    t.maxcode[l] = counts[l - 1] ? code - 1 : -1;
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  if (k != nsym || nsym > 256) return false;
  std::memcpy(t.vals, symbols, nsym);
  // fill the fast table
  code = 0;
  k = 0;
  for (int l = 1; l <= 9; ++l) {
    for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
      const int shift = 9 - l;
      for (int f = 0; f < (1 << shift); ++f) t.fast[(code << shift) | f] = (uint16_t)((l << 8) | t.vals[k]);
    }
    code <<= 1;
  }
  // combined table: every code of length <= FAST_BITS, with the extra bits expanded when they fit
  std::memset(t.comb, 0, sizeof(t.comb));
  std::memset(t.val, 0, sizeof(t.val));
  code = 0;
  k = 0;
  for (int l = 1; l <= FAST_BITS; ++l) {
    for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
      const int sym = t.vals[k], sz = sym & 15, shift = FAST_BITS - l;
      for (int f = 0; f < (1 << shift); ++f) {
        const int idx = (code << shift) | f;
        uint16_t e = (uint16_t)((l << 8) | sym);
        if (l + sz <= FAST_BITS) {
          const int extra = sz ? (f >> (shift - sz)) & ((1 << sz) - 1) : 0;
          t.val[idx] = (int16_t)(sz ? (extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra) : 0);
          e |= (uint16_t)((l + sz) << 12);
        }
        t.comb[idx] = e;
      }
    }
    code <<= 1;
  }
  t.ok = true;
  return true;
}

inline bool has_ff(uint64_t w) {  // any byte == 0xFF
  const uint64_t x = ~w;  // 0xFF -> 0x00
  return ((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) != 0;
}

struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int nbits = 0;
  bool marker = false;  // hit a marker: feed zeros
  int zfill = 0;        // zero bits appended past the data / a marker (the newest bits of acc)
  // the decoder consumed bits that were not in the stream: a truncated (or marker-cut) scan.
  // PIL (no LOAD_TRUNCATED_IMAGES) rejects such a file, so the upload takes that path and fails
  // the same way instead of classifying a grey tail.
  bool overrun() const { return zfill > nbits; }
  void fill() {
    // bulk path: no 0xFF among the next 8 bytes (the usual case) -> one big-endian 64-bit load
    if (!marker && p + 8 <= end) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      if (!has_ff(w)) {
        const int take = (64 - nbits) >> 3;  // whole bytes that fit (fill runs with nbits < 16)
        const uint64_t be = __builtin_bswap64(w);
        acc |= (be >> (64 - 8 * take)) << (64 - 8 * take - nbits);
        p += take;
        nbits += 8 * take;
        return;
      }
    }
    while (nbits <= 56) {
      uint8_t b = 0;
      bool real = false;
      if (!marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          const uint8_t n = p + 1 < end ? p[1] : 0;
          if (n == 0x00) {
            p += 2;
            real = true;
          } else {
            marker = true;  // RSTn / EOI: stop consuming
            b = 0;
          }
        } else {
          ++p;
          real = true;
        }
      }
      if (!real) zfill += 8;
      acc |= (uint64_t)b << (56 - nbits);
      nbits += 8;
    }
  }
  inline uint32_t peek(int n) {
    if (nbits < n) fill();
    return (uint32_t)(acc >> (64 - n));
  }
  inline void skip(int n) {
    acc <<= n;
    nbits -= n;
  }
  inline int get(int n) {
    if (n == 0) return 0;
    const uint32_t v = peek(n);
    skip(n);
    return (int)v;
  }
  void reset_at_marker() {  // byte-align and consume an RSTn marker
    acc = 0;
    nbits = 0;
    zfill = 0;
    marker = false;
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) p += 2;
  }
};

inline int decode_huff(BitReader& br, const Huff& t) {
  const uint32_t look = br.peek(9);
  const uint16_t f = t.fast[look];
  if (f) {
    br.skip(f >> 8);
    return f & 0xFF;
  }
  int code = (int)br.peek(16);
  for (int l = 10; l <= 16; ++l) {
    const int c = code >> (16 - l);
    if (t.maxcode[l] >= 0 && c <= t.maxcode[l] && c >= t.mincode[l]) {
      br.skip(l);
      return t.vals[t.valptr[l] + c - t.mincode[l]];
    }
  }
  return -1;  // corrupt
}

inline int extend(int v, int n) { return v < (1 << (n - 1)) ? v - (1 << n) + 1 : v; }

// JPEG bytes -> container (CONTAINER_BYTES at `out`).  Returns false (with a reason) for anything
// this decoder does not handle; the caller then uses the PIL path.
inline bool jpeg_to_container(const uint8_t* data, size_t n, uint8_t* out, std::string* why = nullptr) {
  auto fail = [&](const char* m) {
    if (why) *why = m;
    return false;
  };
  if (n < 4 || data[0] != 0xFF || data[1] != 0xD8) return fail("not a JPEG");
  uint16_t qt[4][64];
  bool have_q[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  int W = 0, H = 0, nc = 0, restart = 0;
  int cid[3], ch[3], cv[3], cq[3], ctd[3] = {0, 0, 0}, cta[3] = {0, 0, 0};
  bool sof = false;
  size_t i = 2;
  const uint8_t* scan = nullptr;
  while (i + 4 <= n) {
    if (data[i] != 0xFF) return fail("bad marker");
    uint8_t m = data[i + 1];
    if (m == 0xFF) {
      ++i;
      continue;
    }
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7)) {
      i += 2;
      continue;
    }
    if (m == 0xD9) return fail("no scan");
    const size_t len = ((size_t)data[i + 2] << 8) | data[i + 3];
    if (len < 2 || i + 2 + len > n) return fail("truncated segment");
    const uint8_t* seg = data + i + 4;
    const size_t sl = len - 2;
    if (m == 0xDB) {  // DQT
      size_t k = 0;
      while (k < sl) {
        const int pq = seg[k] >> 4, tq = seg[k] & 3;
        ++k;
        if (pq > 1 || k + (pq ? 128 : 64) > sl) return fail("bad DQT");
        for (int j = 0; j < 64; ++j) {
          qt[tq][j] = pq ? (uint16_t)((seg[k + 2 * j] << 8) | seg[k + 2 * j + 1]) : seg[k + j];
        }
        k += pq ? 128 : 64;
        have_q[tq] = true;
      }
    } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1
      if (sl < 6 || seg[0] != 8) return fail("not 8-bit");
      H = (seg[1] << 8) | seg[2];
      W = (seg[3] << 8) | seg[4];
      nc = seg[5];
      if ((nc != 1 && nc != 3) || sl < 6 + 3 * (size_t)nc || W <= 0 || H <= 0) return fail("unsupported components");
      for (int c = 0; c < nc; ++c) {
        cid[c] = seg[6 + 3 * c];
        ch[c] = seg[7 + 3 * c] >> 4;
        cv[c] = seg[7 + 3 * c] & 15;
        cq[c] = seg[8 + 3 * c] & 3;
        if (ch[c] < 1 || ch[c] > 2 || cv[c] < 1 || cv[c] > 2) return fail("sampling factor > 2");
      }
      sof = true;
    } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return fail("progressive / lossless / arithmetic JPEG");
    } else if (m == 0xC4) {  // DHT
      size_t k = 0;
      while (k < sl) {
        if (k + 17 > sl) return fail("bad DHT");
        const int tc = seg[k] >> 4, th = seg[k] & 3;
        int tot = 0;
        for (int j = 0; j < 16; ++j) tot += seg[k + 1 + j];
        if (k + 17 + tot > sl || tc > 1) return fail("bad DHT");
        if (!build_huff(tc ? ac[th] : dc[th], seg + k + 1, seg + k + 17, tot)) return fail("bad Huffman table");
        k += 17 + tot;
      }
    } else if (m == 0xDD) {  // DRI
      if (sl < 2) return fail("bad DRI");
      restart = (seg[0] << 8) | seg[1];
    } else if (m == 0xDA) {  // SOS
      if (!sof) return fail("SOS before SOF");
      const int ns = seg[0];
      if (ns != nc || sl < 1 + 2 * (size_t)ns + 3) return fail("multi-scan JPEG");
      for (int s = 0; s < ns; ++s) {
        const int id = seg[1 + 2 * s];
        int c = 0;
        while (c < nc && cid[c] != id) ++c;
        if (c == nc) return fail("bad scan component");
        ctd[c] = seg[2 + 2 * s] >> 4;
        cta[c] = seg[2 + 2 * s] & 15;
        if (ctd[c] > 3 || cta[c] > 3) return fail("bad table id");
      }
      scan = seg + sl;
      break;
    }
    i += 2 + len;
  }
  if (!scan) return fail("no scan");
  for (int c = 0; c < nc; ++c)
    if (!have_q[cq[c]] || !dc[ctd[c]].ok || !ac[cta[c]].ok) return fail("missing table");

  int hmax = 1, vmax = 1;
  for (int c = 0; c < nc; ++c) {
    hmax = ch[c] > hmax ? ch[c] : hmax;
    vmax = cv[c] > vmax ? cv[c] : vmax;
  }
  const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
  uint32_t nblocks = 0, first[3];
  for (int c = 0; c < nc; ++c) {
    first[c] = nblocks;
    nblocks += (uint32_t)mcux * ch[c] * mcuy * cv[c];
  }
  const size_t groups = ((size_t)nblocks + 63) / 64;
  const size_t counts_off = 384 + 4 * groups, entries_off = (counts_off + nblocks + 1) & ~(size_t)1;
  if (entries_off + 2 * (size_t)nblocks > PAYLOAD_BYTES) return fail("image too large for the container");
  const int pil = [&] {  // PIL draft(): largest d in 8, 4, 2, 1 with d <= min(W // 256, H // 256)
    const int q = (W / IMG_SHORT) < (H / IMG_SHORT) ? W / IMG_SHORT : H / IMG_SHORT;
    for (int d : {8, 4, 2, 1})
      if (q >= d) return d;
    return 1;
  }();
  uint8_t* pay = out + HDR_BYTES;
  // quantised coefficients of every block at full scale (zigzag order), decoded once per image;
  // the encode pass below keeps the s x s corner for the chosen scale
  // the nonzero quantised coefficients of every block (zigzag index + value), decoded once per image
  // in MCU order; the encode pass below walks them in block-table order and keeps those inside the
  // s x s corner of the chosen scale.  Sparse lists instead of a dense 64-per-block buffer: no
  // per-image zeroing, and the encode pass touches only nonzeros (gprof: the dense scan was 57 % of
  // the time on a 320 x 240 q90 photo)
  static thread_local std::vector<uint8_t> czb;
  static thread_local std::vector<int16_t> cvb;
  static thread_local std::vector<uint32_t> boff;
  static thread_local std::vector<uint8_t> bcnt;
  if (czb.size() < (size_t)nblocks * 64) {
    czb.resize((size_t)nblocks * 64);
    cvb.resize((size_t)nblocks * 64);
  }
  if (boff.size() < nblocks) {
    boff.resize(nblocks);
    bcnt.resize(nblocks);
  }
  uint8_t* const zb = czb.data();
  int16_t* const vb = cvb.data();
  uint32_t pos = 0;
  {
    BitReader br{scan, data + n};
    int pred[3] = {0, 0, 0};
    const int total_mcu = mcux * mcuy;
    int todo = restart;
    for (int mcu = 0; mcu < total_mcu; ++mcu) {
      if (restart) {
        if (todo == 0) {
          if (br.overrun()) return fail("truncated scan");
          br.reset_at_marker();
          pred[0] = pred[1] = pred[2] = 0;
          todo = restart;
        }
        --todo;
      }
      const int mx = mcu % mcux, my = mcu / mcux;
      for (int c = 0; c < nc; ++c) {
        const Huff& hdc = dc[ctd[c]];
        const Huff& hac = ac[cta[c]];
        const int bw = mcux * ch[c];
        for (int by = 0; by < cv[c]; ++by)
          for (int bx = 0; bx < ch[c]; ++bx) {
            const size_t bi = (size_t)first[c] + (size_t)(my * cv[c] + by) * bw + mx * ch[c] + bx;
            const uint32_t p0 = pos;
            {  // DC: one combined lookup when code + magnitude bits fit FAST_BITS
              const uint32_t look = br.peek(FAST_BITS);
              const uint16_t e = hdc.comb[look];
              int diff;
              if (e >> 12) {
                if ((e & 0xFF) > 11) return fail("corrupt DC");
                br.skip(e >> 12);
                diff = hdc.val[look];
              } else {
                int t;
                if (e) {
                  br.skip((e >> 8) & 15);
                  t = e & 0xFF;
                } else {
                  t = decode_huff(br, hdc);
                }
                if (t < 0 || t > 11) return fail("corrupt DC");
                diff = t ? extend(br.get(t), t) : 0;
              }
              pred[c] += diff;
              const int dcv = pred[c] > 32767 ? 32767 : pred[c] < -32768 ? -32768 : pred[c];
              if (dcv) {
                zb[pos] = 0;
                vb[pos++] = (int16_t)dcv;
              }
            }
            for (int z = 1; z < 64;) {
              const uint32_t look = br.peek(FAST_BITS);
              const uint16_t e = hac.comb[look];
              int rs, v = 0;
              bool have_v = false;
              if (e >> 12) {
                br.skip(e >> 12);
                rs = e & 0xFF;
                v = hac.val[look];
                have_v = true;
              } else if (e) {
                br.skip((e >> 8) & 15);
                rs = e & 0xFF;
              } else {
                rs = decode_huff(br, hac);
                if (rs < 0) return fail("corrupt AC");
              }
              const int r = rs >> 4, sz = rs & 15;
              if (sz == 0) {
                if (r == 15) {
                  z += 16;
                  continue;
                }
                break;  // EOB
              }
              z += r;
              if (z > 63) return fail("corrupt AC run");
              zb[pos] = (uint8_t)z;
              vb[pos++] = (int16_t)(have_v ? v : extend(br.get(sz), sz));
              ++z;
            }
            boff[bi] = p0;
            bcnt[bi] = (uint8_t)(pos - p0);
          }
      }
    }
    if (br.overrun()) return fail("truncated scan");
  }

  ImgHeader hd;
  std::memset(&hd, 0, sizeof(hd));
  // encode the kept corner at scale d in block-table order; false = does not fit
  auto decode_at = [&](int d, std::string* err) -> bool {
    const int s = 8 / d;
    const size_t w = (size_t)(W + d - 1) / d, hh = (size_t)(H + d - 1) / d;
    if ((size_t)nblocks * s * s + w * hh * 3 + hh * IMG_OUT * 3 > SCRATCH_PER_IMAGE) return *err = "full", false;
    int keep[64];
    for (int z = 0; z < 64; ++z) {
      const int nat = kZigzag[z], r = nat >> 3, cc = nat & 7;
      keep[z] = (r < s && cc < s) ? r * s + cc : -1;
    }
    uint16_t* qtab = reinterpret_cast<uint16_t*>(pay);
    std::memset(qtab, 0, 384);
    for (int c = 0; c < nc; ++c)
      for (int z = 0; z < 64; ++z)
        if (keep[z] >= 0) qtab[c * 64 + keep[z]] = qt[cq[c]][z];
    uint32_t* gstart = reinterpret_cast<uint32_t*>(pay + 384);
    uint8_t* counts = pay + counts_off;
    uint8_t* ent = pay + entries_off;
    const size_t cap_units = (PAYLOAD_BYTES - entries_off) / 2;
    size_t nu = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
      if ((b & 63) == 0) gstart[b >> 6] = (uint32_t)nu;
      const size_t u0 = nu;
      const uint32_t k0 = boff[b], k1 = k0 + bcnt[b];
      for (uint32_t k = k0; k < k1; ++k) {
        const int z = zb[k], v = vb[k];
        if (keep[z] < 0) continue;
        if (v >= -127 && v <= 127) {
          if (nu + 1 > cap_units) return *err = "full", false;
          ent[2 * nu] = (uint8_t)(int8_t)v;
          ent[2 * nu + 1] = (uint8_t)keep[z];
          nu += 1;
        } else {
          if (nu + 2 > cap_units) return *err = "full", false;
          ent[2 * nu] = 0x80;
          ent[2 * nu + 1] = (uint8_t)keep[z];
          ent[2 * nu + 2] = (uint8_t)(v & 0xFF);
          ent[2 * nu + 3] = (uint8_t)((v >> 8) & 0xFF);
          nu += 2;
        }
      }
      counts[b] = (uint8_t)(nu - u0);
    }
    return true;
  };
  int d = pil;
  std::string err;
  while (!decode_at(d, &err)) {
    if (err != "full" || d == 8) return fail(err == "full" ? "image too large for the container" : err.c_str());
    d *= 2;
  }
  const int s = 8 / d;
  hd.magic = IMG_MAGIC;
  hd.kind = KIND_JPEG;
  hd.width = (uint16_t)((W + d - 1) / d);
  hd.height = (uint16_t)((H + d - 1) / d);
  hd.ncomp = (uint8_t)nc;
  hd.s = (uint8_t)s;
  hd.hmax = (uint8_t)hmax;
  hd.vmax = (uint8_t)vmax;
  hd.coarser = d != pil;
  hd.nblocks = nblocks;
  hd.entries_off = (uint32_t)entries_off;
  for (int c = 0; c < nc; ++c) {
    hd.comp[c].h = (uint8_t)ch[c];
    hd.comp[c].v = (uint8_t)cv[c];
    hd.comp[c].bw = (uint16_t)(mcux * ch[c]);
    hd.comp[c].bh = (uint16_t)(mcuy * cv[c]);
    hd.comp[c].offset = first[c];
  }
  if (!fill_geometry(hd)) return fail("aspect ratio beyond the container's resize range");
  std::memcpy(out, &hd, sizeof(hd));
  return true;
}

}  // namespace mlsjpeg
