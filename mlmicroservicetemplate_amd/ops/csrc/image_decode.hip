// Device half of the GPU JPEG path: image containers (frontend/csrc/jpeg_coefs.h;
// a raw 224 x 224 x 3 upload, or the Huffman-decoded, dequantised, sparse DCT coefficients of a
// baseline JPEG) -> the model's uint8 [B, 224, 224, 3] input, as the first kernels of the serving
// graph.  ops/image_reference.py is the step-for-step specification (and the test oracle):
//   1. idct:   one 64-lane slot per DCT block: scatter the block's entries into LDS, separable
//              s x s IDCT in fp64 (s = 8 / the DCT downscale), + 128, round, clamp -> component plane
//   2. color:  per pixel: libjpeg-turbo's chroma upsampling (fancy h2v1 / h2v2 triangle filters,
//              replication otherwise) and its 16-bit fixed-point YCbCr -> RGB
//   3. hpass / vpass: Pillow's BILINEAR resample of decode_image (shorter side 256, support scaled
//              by the downscale factor, 22-bit fixed-point weights, each pass rounded to uint8),
//              evaluated only on the 224 x 224 centre crop; raw containers are copied through.
// Scratch per image (planes, RGB, the horizontal pass) lives in one device buffer sized by the
// caller; every index is checked against the header's sizes so a corrupt container cannot write
// outside its image's scratch.
#include "common.h"

namespace {

constexpr int IMG_HDR = 64;
constexpr int IMG_OUT = 224;
constexpr long IMG_PAYLOAD = (long)IMG_OUT * IMG_OUT * 3;
constexpr long IMG_CONTAINER = IMG_HDR + IMG_PAYLOAD;
constexpr uint32_t IMG_MAGIC = 0x4A534C4Du;
constexpr int PRECISION_BITS = 32 - 8 - 2;

struct Hdr {
  uint32_t kind;
  int W, H, nc, s, hmax, vmax;
  int ch[3], cv[3], bw[3], bh[3], first[3];
  int rw, rh, left, top;
  uint32_t nblocks, entries_off;
  bool ok;
};

MLS_DEV uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
MLS_DEV int rd16(const uint8_t* p) { return p[0] | (p[1] << 8); }

MLS_DEV Hdr parse(const uint8_t* c0, long scratch_per_image) {
  // the 64-B header in four 16-B loads (the container base is 16-B aligned), every field picked from
  // those registers at a constant offset: ~40 byte loads per thread before, and no private array
  const uint4* p4 = reinterpret_cast<const uint4*>(c0);
  const uint4 q[4] = {p4[0], p4[1], p4[2], p4[3]};
  auto b8 = [&](int off) -> int {
    const uint4 v = q[off >> 4];
    const int w = (off >> 2) & 3;
    const uint32_t d = w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
    return (int)((d >> (8 * (off & 3))) & 0xFF);
  };
  auto r16 = [&](int off) { return b8(off) | (b8(off + 1) << 8); };
  auto r32 = [&](int off) { return (uint32_t)r16(off) | ((uint32_t)r16(off + 2) << 16); };
  Hdr h;
  h.ok = r32(0) == IMG_MAGIC;
  h.kind = r32(4);
  h.W = r16(8);
  h.H = r16(10);
  h.nc = b8(12);
  h.s = b8(13);
  h.hmax = b8(14);
  h.vmax = b8(15);
  long plane_px = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int o = 16 + 10 * i;
    h.ch[i] = b8(o);
    h.cv[i] = b8(o + 1);
    h.bw[i] = r16(o + 2);
    h.bh[i] = r16(o + 4);
    h.first[i] = (int)r32(o + 6);
    if (i < h.nc) plane_px += (long)h.bw[i] * h.bh[i] * h.s * h.s;
  }
  h.rw = r16(46);
  h.rh = r16(48);
  h.left = r16(50);
  h.top = r16(52);
  h.nblocks = r32(55);
  h.entries_off = r32(59);
  if (h.kind == 1) {
    const bool sgood = h.s == 1 || h.s == 2 || h.s == 4 || h.s == 8;
    const long need = plane_px + (long)h.W * h.H * 3 + (long)h.H * IMG_OUT * 3;
    h.ok = h.ok && sgood && (h.nc == 1 || h.nc == 3) && h.W > 0 && h.H > 0 && h.hmax >= 1 && h.vmax >= 1 &&
           need <= scratch_per_image && h.rw >= IMG_OUT && h.rh >= IMG_OUT && h.left + IMG_OUT <= h.rw &&
           h.top + IMG_OUT <= h.rh && 384 + 4 * (((long)h.nblocks + 63) / 64) + (long)h.nblocks <= (long)h.entries_off &&
           h.entries_off <= IMG_PAYLOAD;
#pragma unroll
    for (int i = 0; i < 3; ++i)  // constant indices: the header stays in registers
      if (i < h.nc)
        h.ok = h.ok && h.ch[i] >= 1 && h.cv[i] >= 1 && (long)h.first[i] + (long)h.bw[i] * h.bh[i] <= (long)h.nblocks &&
               h.bw[i] * h.s >= (h.W * h.ch[i] + h.hmax - 1) / h.hmax &&
               h.bh[i] * h.s >= (h.H * h.cv[i] + h.vmax - 1) / h.vmax;
  }
  return h;
}

// scratch layout per image: planes (component-major), then RGB [H][W][3], then hpass [H][224][3]
// component-indexed header fields with a runtime index, kept in registers (a dynamically indexed
// struct array goes to scratch memory)
MLS_DEV int at3(const int (&a)[3], int i) { return i == 0 ? a[0] : i == 1 ? a[1] : a[2]; }

MLS_DEV long plane_off(const Hdr& h, int comp) {
  long o = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < comp) o += (long)h.bw[i] * h.bh[i] * h.s * h.s;
  return o;
}
MLS_DEV long rgb_off(const Hdr& h) { return plane_off(h, h.nc); }
MLS_DEV long hp_off(const Hdr& h) { return rgb_off(h) + (long)h.W * h.H * 3; }

// ---- 1. IDCT: 4 blocks per 256-thread workgroup, one 64-lane wave each (grid-stride over the
// image's blocks: the launch geometry is fixed, so it can be captured once for any container).
// Entry parsing is wave-parallel: the block's first unit = its group's start + an in-wave sum of the
// group's earlier counts (one coalesced byte load per lane); each lane takes one 2-byte unit, and
// the rare escapes (0x80 marker + an int16 in the next unit) are resolved on the ballot mask of
// marker candidates -- a lane-0 scan of up to 63 counts and every entry (dependent byte loads)
// measured ~70 % of this kernel before ----
constexpr int IDCT_WG = 64;  // workgroups per image
__global__ __launch_bounds__(256) void img_idct_kernel(const uint8_t* __restrict__ cont, uint8_t* __restrict__ scratch,
                                                       long scratch_per_image) {
  const int b = blockIdx.y;
  const uint8_t* c = cont + (long)b * IMG_CONTAINER;
  __shared__ double F[4][64];
  __shared__ double T[4][64];
  __shared__ double Mc[64];  // IDCT basis of this image's scale: Mc[x * s + u] = c(u)/2 cos((2x+1)u pi / 2s)
  const Hdr h = parse(c, scratch_per_image);
  if (!h.ok || h.kind != 1) return;
  const int slot = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int s = h.s, ss = s * s;
  const int y = t / s, x = t - y * s;  // pass 1: thread = (v, x); pass 2: (y, x)
  const double PI = 3.14159265358979323846;
  if (threadIdx.x < ss) {  // once per workgroup, not once per multiply (fp64 cos is a long software routine)
    const int xx = threadIdx.x / s, uu = threadIdx.x - xx * s;
    Mc[threadIdx.x] = (uu == 0 ? 0.70710678118654752440 : 1.0) * 0.5 * cos((2 * xx + 1) * uu * PI / (2 * s));
  }
  uint8_t* sc = scratch + (long)b * scratch_per_image;
  const uint8_t* pay = c + IMG_HDR;
  const long groups = ((long)h.nblocks + 63) / 64, counts_off = 384 + 4 * groups;
  const long cap = (IMG_PAYLOAD - (long)h.entries_off) / 2;  // units that fit the container
  const uint8_t* ent = pay + h.entries_off;
  const long stride = (long)gridDim.x * 4;
  for (long base = (long)blockIdx.x * 4; base < (long)h.nblocks; base += stride) {  // uniform per workgroup
    const long blk = base + slot;
    const bool live = blk < (long)h.nblocks;  // uniform per wave
    F[slot][t] = 0.0;
    const int comp = (h.nc > 2 && blk >= h.first[2]) ? 2 : (h.nc > 1 && blk >= h.first[1]) ? 1 : 0;
    __syncthreads();
    if (live) {
      const long g = blk >> 6;
      const int k = (int)(blk & 63);
      // units before this block in its group: sum of counts[g*64 + L] over lanes L < k
      int before = t < k ? pay[counts_off + g * 64 + t] : 0;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) before += __shfl_xor(before, o);
      const long u0 = (long)rd32(pay + 384 + 4 * g) + before;
      const int n = pay[counts_off + blk];
      bool carry = false;  // the previous chunk ended on a marker: this chunk's unit 0 is its payload
      for (int c0 = 0; c0 < n; c0 += 64) {
        const long u = u0 + c0 + t;
        const bool in = c0 + t < n && u < cap;
        const int b0 = in ? ent[2 * u] : 0, b1 = in ? ent[2 * u + 1] : 0;
        // true markers among the candidates (a payload unit is never a marker): scan the set bits
        unsigned long long cand = __ballot(in && b0 == 0x80), mk = 0;
        if (carry) cand &= ~1ull;
        while (cand) {
          const int q = __builtin_ctzll(cand);
          mk |= 1ull << q;
          cand &= q >= 62 ? 0ull : ~0ull << (q + 2);
        }
        const bool is_payload = t == 0 ? carry : ((mk >> (t - 1)) & 1) != 0;
        const bool is_marker = (mk >> t) & 1;
        // the escape's int16 sits in the next unit -- held by lane t + 1 (chunk tail: read it)
        const int nb0 = __shfl_down(b0, 1), nb1 = __shfl_down(b1, 1);
        int v;
        if (is_marker) {
          v = t < 63 ? (int)(int16_t)(nb0 | (nb1 << 8))
                     : (u + 1 < cap ? (int)(int16_t)(ent[2 * (u + 1)] | (ent[2 * (u + 1) + 1] << 8)) : 0);
        } else {
          v = (int)(int8_t)b0;
        }
        const int pos = b1;
        if (in && !is_payload && pos < ss)
          F[slot][pos] = (double)v * (double)rd16(pay + 2 * (comp * 64 + pos));
        carry = (mk >> 63) & 1;
      }
    }
    __syncthreads();
    if (live && t < ss) {  // T[v][x] = sum_u F[v][u] M[x][u]
      double acc = 0.0;
      for (int u = 0; u < s; ++u) acc += F[slot][y * s + u] * Mc[x * s + u];
      T[slot][t] = acc;
    }
    __syncthreads();
    if (live && t < ss) {
      double acc = 0.0;  // P[y][x] = sum_v M[y][v] T[v][x]
      for (int v = 0; v < s; ++v) acc += Mc[y * s + v] * T[slot][v * s + x];
      int px = (int)floor(acc + 128.0 + 0.5);
      px = px < 0 ? 0 : px > 255 ? 255 : px;
      const int bwc = at3(h.bw, comp);
      const long local = blk - at3(h.first, comp);
      const int row = (int)(local / bwc), col = (int)(local - (long)row * bwc);
      if (row < at3(h.bh, comp)) {
        const long pw = (long)bwc * s;
        sc[plane_off(h, comp) + (long)(row * s + y) * pw + col * s + x] = (uint8_t)px;
      }
    }
    __syncthreads();  // T / F reused by the next round
  }
}

MLS_DEV int fix16(double x) { return (int)(x * 65536.0 + 0.5); }

// chroma sample (component `cc`) at full-resolution pixel (y, x): libjpeg's upsampling
MLS_DEV int chroma(const uint8_t* pl, const Hdr& h, int cc, int y, int x) {
  const int fx = h.hmax / h.ch[cc], fy = h.vmax / h.cv[cc];
  const int cw = (h.W * h.ch[cc] + h.hmax - 1) / h.hmax, chh = (h.H * h.cv[cc] + h.vmax - 1) / h.vmax;
  const long pw = (long)h.bw[cc] * h.s;
  if (fx == 1 && fy == 1) return pl[(long)y * pw + x];
  if (fx == 2 && fy == 1 && h.s > 1) {
    const uint8_t* r = pl + (long)y * pw;
    const int c = x >> 1, n = cw;
    if ((x & 1) == 0) return c == 0 ? r[0] : (3 * r[c] + r[c - 1] + 1) >> 2;
    return c == n - 1 ? r[n - 1] : (3 * r[c] + r[c + 1] + 2) >> 2;
  }
  if (fx == 2 && fy == 2 && h.s > 1) {
    const int cy = y >> 1, nbr = (y & 1) == 0 ? (cy > 0 ? cy - 1 : 0) : (cy + 1 < chh ? cy + 1 : chh - 1);
    const uint8_t* r0 = pl + (long)cy * pw;
    const uint8_t* r1 = pl + (long)nbr * pw;
    const int c = x >> 1, n = cw;
    auto tcol = [&](int k) { return 3 * r0[k] + r1[k]; };
    if ((x & 1) == 0) return c == 0 ? (4 * tcol(0) + 8) >> 4 : (3 * tcol(c) + tcol(c - 1) + 8) >> 4;
    return c == n - 1 ? (4 * tcol(n - 1) + 7) >> 4 : (3 * tcol(c) + tcol(c + 1) + 7) >> 4;
  }
  const int yy = y / fy < chh ? y / fy : chh - 1, xx = x / fx < cw ? x / fx : cw - 1;
  return pl[(long)yy * pw + xx];
}

// ---- 2. upsampling + colour conversion -> RGB [H][W][3] ----
__global__ __launch_bounds__(256) void img_color_kernel(const uint8_t* __restrict__ cont, uint8_t* __restrict__ scratch,
                                                        long scratch_per_image) {
  const int b = blockIdx.y;
  const uint8_t* c = cont + (long)b * IMG_CONTAINER;
  const Hdr h = parse(c, scratch_per_image);
  if (!h.ok || h.kind != 1) return;
  const long n = (long)h.W * h.H;
  uint8_t* sc = scratch + (long)b * scratch_per_image;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < (int)n; i += gridDim.x * 256) {
    const int y = i / h.W, x = i - y * h.W;
    const uint8_t* p0 = sc + plane_off(h, 0);
    const int Y = p0[(long)y * h.bw[0] * h.s + x];
    int r, g, bb;
    if (h.nc == 1) {
      r = g = bb = Y;
    } else {
      const int cb = chroma(sc + plane_off(h, 1), h, 1, y, x) - 128;
      const int cr = chroma(sc + plane_off(h, 2), h, 2, y, x) - 128;
      r = Y + ((fix16(1.40200) * cr + (1 << 15)) >> 16);
      g = Y + ((-fix16(0.34414) * cb - fix16(0.71414) * cr + (1 << 15)) >> 16);
      bb = Y + ((fix16(1.77200) * cb + (1 << 15)) >> 16);
    }
    uint8_t* o = sc + rgb_off(h) + i * 3;
    o[0] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
    o[1] = (uint8_t)(g < 0 ? 0 : g > 255 ? 255 : g);
    o[2] = (uint8_t)(bb < 0 ? 0 : bb > 255 ? 255 : bb);
  }
}

// Pillow precompute_coeffs (bilinear) for output index xx: first source index, taps, fixed weights
constexpr int MAX_TAPS = 33;
template <int KSTRIDE = 1>  // kk[j * KSTRIDE]: 1 for one set, IMG_OUT for the hpass's per-column sets in LDS
MLS_DEV int pil_coeffs(int in_size, int out_size, int xx, int* kk) {
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > MAX_TAPS) xmax = MAX_TAPS;
  // two passes recomputing the triangle weight (no local double array: it would live in scratch)
  auto tri = [&](int x) {
    double t = (x + xmin - center + 0.5) * ss;
    t = t < 0 ? -t : t;
    return t < 1.0 ? 1.0 - t : 0.0;
  };
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += tri(x);
  for (int x = 0; x < xmax; ++x) {
    const double k = tri(x);
    const double v = (ww != 0.0 ? k / ww : k) * (double)(1 << PRECISION_BITS);
    kk[x * KSTRIDE] = v < 0 ? (int)(v - 0.5) : (int)(v + 0.5);
  }
  kk[(MAX_TAPS - 1) * KSTRIDE] = xmax;  // tap count rides in the last slot
  return xmin;
}

MLS_DEV uint8_t clip8(long v) {
  v >>= PRECISION_BITS;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// ---- 3. horizontal pass over the crop's 224 columns: [H][224][3]; workgroup x takes rows x, x + G, ... ----
__global__ __launch_bounds__(256) void img_hpass_kernel(const uint8_t* __restrict__ cont, uint8_t* __restrict__ scratch,
                                                        long scratch_per_image) {
  const int b = blockIdx.y;
  const uint8_t* c = cont + (long)b * IMG_CONTAINER;
  const Hdr h = parse(c, scratch_per_image);
  if (!h.ok || h.kind != 1) return;
  uint8_t* sc = scratch + (long)b * scratch_per_image;
  const uint8_t* rgb = sc + rgb_off(h);
  uint8_t* hp = sc + hp_off(h);
  const int ox = threadIdx.x;
  if (ox >= IMG_OUT) return;
  const int x = h.left + ox;
  if (h.rw == h.W) {
    for (int y = blockIdx.x; y < h.H; y += gridDim.x)
      for (int ch = 0; ch < 3; ++ch) hp[((long)y * IMG_OUT + ox) * 3 + ch] = rgb[((long)y * h.W + x) * 3 + ch];
    return;
  }
  // this column's taps in LDS ([tap][column]: lanes read consecutive words), not a per-thread array
  // (dynamically indexed -> scratch memory)
  __shared__ int kks[MAX_TAPS * IMG_OUT];
  int* kk = kks + ox;
  const int xmin = pil_coeffs<IMG_OUT>(h.W, h.rw, x, kk);
  const int taps = kk[(MAX_TAPS - 1) * IMG_OUT];
  for (int y = blockIdx.x; y < h.H; y += gridDim.x) {
    long a0 = 1L << (PRECISION_BITS - 1), a1 = a0, a2 = a0;
    const uint8_t* r = rgb + ((long)y * h.W + xmin) * 3;
    for (int j = 0; j < taps; ++j) {
      const long w = kk[j * IMG_OUT];
      a0 += (long)r[3 * j] * w;
      a1 += (long)r[3 * j + 1] * w;
      a2 += (long)r[3 * j + 2] * w;
    }
    uint8_t* o = hp + ((long)y * IMG_OUT + ox) * 3;
    o[0] = clip8(a0);
    o[1] = clip8(a1);
    o[2] = clip8(a2);
  }
}

// ---- 4. vertical pass over the crop's 224 rows -> out [224][224][3]; raw containers copied ----
__global__ __launch_bounds__(256) void img_vpass_kernel(const uint8_t* __restrict__ cont, uint8_t* __restrict__ scratch,
                                                        long scratch_per_image, uint8_t* __restrict__ out, int* err) {
  const int b = blockIdx.y;
  const uint8_t* c = cont + (long)b * IMG_CONTAINER;
  uint8_t* o = out + (long)b * IMG_PAYLOAD;
  const Hdr h = parse(c, scratch_per_image);
  const int oy = blockIdx.x;  // one output row per workgroup
  const bool bad = !h.ok || (h.kind != 0 && h.kind != 1);
  if (threadIdx.x == 0 && oy == 0 && err) err[b] = bad ? 1 : 0;  // per image: every row written each launch
  if (bad) {  // unusable container: a black image + its error flag
    for (int i = threadIdx.x; i < IMG_OUT * 3; i += 256) o[(long)oy * IMG_OUT * 3 + i] = 0;
    return;
  }
  if (h.kind == 0) {  // a row is 672 B = 42 x 16 B; the container payload starts 64-B aligned
    const uint4* src = reinterpret_cast<const uint4*>(c + IMG_HDR + (long)oy * IMG_OUT * 3);
    uint4* dst = reinterpret_cast<uint4*>(o + (long)oy * IMG_OUT * 3);
    if (threadIdx.x < IMG_OUT * 3 / 16) dst[threadIdx.x] = src[threadIdx.x];
    return;
  }
  const uint8_t* hp = scratch + (long)b * scratch_per_image + hp_off(h);
  const int y = h.top + oy;
  if (h.rh == h.H) {
    for (int i = threadIdx.x; i < IMG_OUT * 3; i += 256) o[(long)oy * IMG_OUT * 3 + i] = hp[(long)y * IMG_OUT * 3 + i];
    return;
  }
  __shared__ int kk[MAX_TAPS];
  __shared__ int ymin;
  if (threadIdx.x == 0) ymin = pil_coeffs(h.H, h.rh, y, kk);
  __syncthreads();
  const int taps = kk[MAX_TAPS - 1];
  for (int i = threadIdx.x; i < IMG_OUT * 3; i += 256) {
    long a = 1L << (PRECISION_BITS - 1);
    for (int j = 0; j < taps; ++j) a += (long)hp[(long)(ymin + j) * IMG_OUT * 3 + i] * kk[j];
    o[(long)oy * IMG_OUT * 3 + i] = clip8(a);
  }
}

}  // namespace

extern "C" {

// containers [B][64 + 224*224*3] uint8 -> out [B][224][224][3] uint8.  scratch: B * scratch_per_image
// bytes (planes + RGB + the horizontal pass of one image; a container needing more is reported).
// err (nullable): int32 [B], err[b] = 1 when container b is unusable (that image comes out black), else 0
// (written every launch: no clearing needed inside a graph).  Fixed launch
// geometry (grid-stride loops), so one captured graph serves any mix of containers.
int mls_image_decode(const void* cont, void* out, void* scratch, long scratch_per_image, int B, int* err,
                     void* stream) {
  if (B <= 0 || scratch_per_image <= 0) return MLS_BAD_ARG;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* c = (const uint8_t*)cont;
  uint8_t* sc = (uint8_t*)scratch;
  hipLaunchKernelGGL(img_idct_kernel, dim3(IDCT_WG, B), dim3(256), 0, st, c, sc, scratch_per_image);
  hipLaunchKernelGGL(img_color_kernel, dim3(64, B), dim3(256), 0, st, c, sc, scratch_per_image);
  hipLaunchKernelGGL(img_hpass_kernel, dim3(16, B), dim3(256), 0, st, c, sc, scratch_per_image);
  hipLaunchKernelGGL(img_vpass_kernel, dim3(IMG_OUT, B), dim3(256), 0, st, c, sc, scratch_per_image, (uint8_t*)out,
                     err);
  return (int)hipGetLastError();
}

}  // extern "C"
