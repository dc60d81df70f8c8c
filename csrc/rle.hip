// COCO run-length encoding of instance masks on the GPU, and batched mask IoU from the encoded form (SURVEY §2.10
// K23; reference detection/mean_ap.py:790-821 encodes every mask on the host with pycocotools, one call per mask,
// and COCOeval computes mask IoU per image from the RLE strings).
//
// Encode (``rle_encode``; masks [K, H, W], any nonzero = foreground):
//   1. change words — a block stages a 64 x 64 pixel tile through LDS (coalesced row loads) and each of its first 64
//      threads turns one column of the tile into a 64-bit word in COLUMN-MAJOR pixel order (COCO's order), XORed
//      with itself shifted by one pixel: bit b is set where pixel x H + 64 wy + b differs from its predecessor
//      (pixel 0's predecessor is background, so a mask starting with foreground gets COCO's leading empty run);
//   2. per-mask exclusive scan of the words' popcounts (ATen cumsum) -> every change's index; one host read of the
//      per-mask change counts sizes the outputs;
//   3. change positions written by their word's thread; run i of mask k = [P[i - 1], P[i]) (0 and H W at the ends);
//   4. COCO's compressed counts string (``rleToString``: 5-bit groups + 48, continuation bit 0x20, sign bit 0x10,
//      run i > 2 stored as the difference to run i - 2): one thread per run sizes its characters, a scan places them,
//      the same thread writes them.  Only the strings travel to the host (the masks never do).
// Decode for IoU (``rle_decode_bits``): one thread per mask parses its string into cumulative run ends; one thread
// per 64-pixel word binary-searches the run covering its first pixel and fills the word (column-major bits, the
// layout both sides of an IoU share).  ``mask_iou_tiles``: 16 x 16 (detection, ground truth) tiles of ALL images in
// one launch (tile list built on the host), popcount(d & g) over LDS-staged 64-word chunks — the per-image launch
// loop of the dense-mask path is gone.
// CPU implementations of the same three ops give identical bytes / values (host evaluator, CPU states).
#include "common.h"

#include <ATen/Parallel.h>

namespace tmx {

constexpr int kRleTile = 64;

// chg[k][x][wy] (WY = ceil(H / 64) words per column) and its popcount
__global__ void __launch_bounds__(256) rle_change_kernel(const uint8_t* __restrict__ masks, int64_t H, int64_t W, int WY, int64_t k0,
                                                         uint64_t* __restrict__ chg, int32_t* __restrict__ cnt) {
  __shared__ uint8_t tile[kRleTile][kRleTile + 4];
  const int64_t x0 = (int64_t)blockIdx.x * kRleTile;
  const int wy = blockIdx.y;
  const int64_t y0 = (int64_t)wy * kRleTile;
  const int64_t k = k0 + blockIdx.z;
  const uint8_t* m = masks + k * H * W;
  for (int e = threadIdx.x; e < kRleTile * kRleTile; e += 256) {
    const int r = e / kRleTile, c = e % kRleTile;
    const int64_t y = y0 + r, x = x0 + c;
    tile[r][c] = (y < H && x < W) ? (m[y * W + x] != 0 ? 1 : 0) : 0;
  }
  __syncthreads();
  if (threadIdx.x >= kRleTile) return;
  const int64_t x = x0 + threadIdx.x;
  if (x >= W) return;
  const int nrows = static_cast<int>(min<int64_t>(kRleTile, H - y0));
  uint64_t w = 0;
  for (int r = 0; r < nrows; ++r) w |= static_cast<uint64_t>(tile[r][threadIdx.x]) << r;
  uint64_t prev = 0;
  if (y0 > 0) prev = m[(y0 - 1) * W + x] != 0 ? 1 : 0;
  else if (x > 0) prev = m[(H - 1) * W + x - 1] != 0 ? 1 : 0;
  uint64_t c = w ^ ((w << 1) | prev);
  if (nrows < 64) c &= (uint64_t{1} << nrows) - 1;
  const int64_t o = (k * W + x) * WY + wy;
  chg[o] = c;
  cnt[o] = __popcll(c);
}

// change positions: word o of mask k writes its changes at P[pbase[k] + excl[o] ...]
__global__ void __launch_bounds__(256) rle_positions_kernel(const uint64_t* __restrict__ chg, const int64_t* __restrict__ excl,
                                                            const int64_t* __restrict__ pbase, int64_t words_per_mask, int64_t total_words,
                                                            int64_t H, int WY, int32_t* __restrict__ P) {
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total_words; o += (int64_t)gridDim.x * blockDim.x) {
    uint64_t c = chg[o];
    if (!c) continue;
    const int64_t k = o / words_per_mask, wi = o % words_per_mask;
    const int64_t x = wi / WY, wy = wi % WY;
    int64_t j = pbase[k] + excl[o];
    const int64_t base = x * H + wy * 64;
    while (c) {
      const int b = __ffsll(static_cast<unsigned long long>(c)) - 1;
      P[j++] = static_cast<int32_t>(base + b);
      c &= c - 1;
    }
  }
}

__device__ __forceinline__ int64_t rle_run_len(const int32_t* __restrict__ P, int64_t pb, int64_t m, int64_t HW, int64_t i) {
  const int64_t s = i == 0 ? 0 : P[pb + i - 1];
  const int64_t e = i == m ? HW : P[pb + i];
  return e - s;
}

// one thread per run g (global): mask k by binary search in rbase[K + 1]; WRITE = false sizes the characters
template <bool WRITE>
__global__ void __launch_bounds__(256) rle_chars_kernel(const int32_t* __restrict__ P, const int64_t* __restrict__ pbase,
                                                        const int64_t* __restrict__ rbase, int K, int64_t HW, int64_t R,
                                                        int32_t* __restrict__ lens, const int64_t* __restrict__ coff,
                                                        uint8_t* __restrict__ out) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < R; g += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = K;  // last k with rbase[k] <= g
    while (hi - lo > 1) {
      const int mid = (lo + hi) / 2;
      if (rbase[mid] <= g) lo = mid; else hi = mid;
    }
    const int k = lo;
    const int64_t i = g - rbase[k];
    const int64_t pb = pbase[k], m = pbase[k + 1] - pb;
    long long x = rle_run_len(P, pb, m, HW, i);
    if (i > 2) x -= rle_run_len(P, pb, m, HW, i - 2);
    int nc = 0;
    bool more = true;
    int64_t o = WRITE ? coff[g] : 0;
    while (more) {
      int c = static_cast<int>(x & 0x1f);
      x >>= 5;
      more = (c & 0x10) ? x != -1 : x != 0;
      if (more) c |= 0x20;
      if (WRITE) out[o + nc] = static_cast<uint8_t>(c + 48);
      ++nc;
    }
    if (!WRITE) lens[g] = nc;
  }
}

std::tuple<at::Tensor, at::Tensor> rle_encode_cuda(const at::Tensor& masks_in) {
  TORCH_CHECK(masks_in.dim() == 3, "rle_encode: expected [K, H, W] masks");
  const at::DeviceGuard guard(masks_in.device());
  auto masks = (masks_in.scalar_type() == at::kBool || masks_in.scalar_type() == at::kByte ? masks_in : masks_in.ne(0)).contiguous();
  const int64_t K = masks.size(0), H = masks.size(1), W = masks.size(2), HW = H * W;
  TORCH_CHECK(HW < (int64_t{1} << 31), "rle_encode: more than 2^31 pixels per mask");
  auto opts = masks.options();
  auto cpu_i64 = at::TensorOptions().dtype(at::kLong);
  if (K == 0) return {at::empty({0}, at::TensorOptions().dtype(at::kByte)), at::zeros({1}, cpu_i64)};
  const int WY = static_cast<int>((H + 63) / 64);
  const int64_t wpm = W * WY, total_words = K * wpm;
  at::Tensor m_dev;
  at::Tensor chg, excl;
  if (HW > 0) {
    chg = at::empty({total_words}, opts.dtype(at::kLong));
    auto cnt = at::empty({total_words}, opts.dtype(at::kInt));
    for (int64_t k0 = 0; k0 < K; k0 += 65535) {  // grid z <= 65535 masks per launch
      dim3 grid(static_cast<unsigned>((W + kRleTile - 1) / kRleTile), static_cast<unsigned>(WY),
                static_cast<unsigned>(std::min<int64_t>(65535, K - k0)));
      hipLaunchKernelGGL(rle_change_kernel, grid, 256, 0, stream(), reinterpret_cast<const uint8_t*>(masks.data_ptr()), H, W, WY, k0,
                         reinterpret_cast<uint64_t*>(chg.data_ptr<int64_t>()), cnt.data_ptr<int32_t>());
      TMX_LAUNCH_CHECK();
    }
    auto cnt64 = cnt.view({K, wpm}).to(at::kLong);
    auto cs = cnt64.cumsum(1);
    m_dev = cs.select(1, wpm - 1).contiguous();
    excl = (cs - cnt64).contiguous();
  } else {
    m_dev = at::zeros({K}, opts.dtype(at::kLong));
  }
  auto pbase = at::cat({at::zeros({1}, m_dev.options()), m_dev.cumsum(0)});
  const int64_t M = pbase[K].item<int64_t>();  // the one size read of the change pass
  const int64_t R = M + K;
  auto rbase = pbase + at::arange(K + 1, pbase.options());
  auto P = at::empty({std::max<int64_t>(M, 1)}, opts.dtype(at::kInt));
  if (M > 0) {
    hipLaunchKernelGGL(rle_positions_kernel, grid_for(total_words, 256, 8192), 256, 0, stream(),
                       reinterpret_cast<const uint64_t*>(chg.data_ptr<int64_t>()), excl.data_ptr<int64_t>(), pbase.data_ptr<int64_t>(),
                       wpm, total_words, H, WY, P.data_ptr<int32_t>());
    TMX_LAUNCH_CHECK();
  }
  auto lens = at::empty({R}, opts.dtype(at::kInt));
  const dim3 rgrid = grid_for(R, 256, 8192);
  hipLaunchKernelGGL((rle_chars_kernel<false>), rgrid, 256, 0, stream(), P.data_ptr<int32_t>(), pbase.data_ptr<int64_t>(),
                     rbase.data_ptr<int64_t>(), static_cast<int>(K), HW, R, lens.data_ptr<int32_t>(), nullptr, nullptr);
  TMX_LAUNCH_CHECK();
  auto incl = lens.to(at::kLong).cumsum(0);
  auto coff = (incl - lens).contiguous();
  auto moff = at::cat({coff.index_select(0, rbase.slice(0, 0, K)), incl.slice(0, R - 1, R)}).cpu();
  const int64_t total = moff[K].item<int64_t>();
  auto chars = at::empty({total}, opts.dtype(at::kByte));
  hipLaunchKernelGGL((rle_chars_kernel<true>), rgrid, 256, 0, stream(), P.data_ptr<int32_t>(), pbase.data_ptr<int64_t>(),
                     rbase.data_ptr<int64_t>(), static_cast<int>(K), HW, R, nullptr, coff.data_ptr<int64_t>(),
                     chars.data_ptr<uint8_t>());
  TMX_LAUNCH_CHECK();
  return {chars.cpu(), moff};
}

// ------------------------------------------------------------------------------------------------------ decode
// one thread per mask: cumulative run ends B_j (int32) at bnd[coff[k] + j] (a string of L chars has <= L runs)
__global__ void __launch_bounds__(64) rle_parse_kernel(const uint8_t* __restrict__ chars, const int64_t* __restrict__ coff, int K,
                                                       int32_t* __restrict__ bnd, int32_t* __restrict__ nrun, double* __restrict__ area) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int64_t b = coff[k], e = coff[k + 1];
  int64_t p = b;
  int j = 0;
  long long c1 = 0, c2 = 0;  // runs j - 1, j - 2
  long long end = 0, fg = 0;
  while (p < e) {
    long long x = 0;
    int sh = 0;
    bool more = true;
    while (more && p < e) {
      const int c = static_cast<int>(chars[p++]) - 48;
      x |= static_cast<long long>(c & 0x1f) << sh;
      more = (c & 0x20) != 0;
      sh += 5;
      if (!more && (c & 0x10)) x |= -1ll << sh;
    }
    if (j > 2) x += c2;
    end += x;
    if (j & 1) fg += x;
    bnd[b + j] = static_cast<int32_t>(end);
    c2 = c1;
    c1 = x;
    ++j;
  }
  nrun[k] = j;
  area[k] = static_cast<double>(fg);
}

__global__ void __launch_bounds__(256) rle_fill_kernel(const int32_t* __restrict__ bnd, const int64_t* __restrict__ coff,
                                                       const int32_t* __restrict__ nrun, int64_t HW, int64_t words, int64_t total,
                                                       uint64_t* __restrict__ bits) {
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = o / words, w = o % words;
    const int32_t* B = bnd + coff[k];
    const int n = nrun[k];
    const int64_t lo = w * 64, hi = min<int64_t>(lo + 64, HW);
    int a = 0, z = n;  // first run j with B_j > lo
    while (a < z) {
      const int mid = (a + z) / 2;
      if (B[mid] > lo) z = mid; else a = mid + 1;
    }
    uint64_t word = 0;
    int64_t start = a == 0 ? 0 : B[a - 1];
    for (int j = a; j < n && start < hi; ++j) {
      const int64_t e = B[j];
      if ((j & 1) && e > lo) {
        const int64_t s0 = max(start, lo), e0 = min(e, hi);
        if (e0 > s0) {
          const int nb = static_cast<int>(e0 - s0);
          const uint64_t run = nb == 64 ? ~uint64_t{0} : ((uint64_t{1} << nb) - 1);
          word |= run << (s0 - lo);
        }
      }
      start = e;
    }
    bits[o] = word;
  }
}

std::tuple<at::Tensor, at::Tensor> rle_decode_bits_cuda(const at::Tensor& chars_in, const at::Tensor& coff_in, int64_t H, int64_t W) {
  const at::DeviceGuard guard(chars_in.device());
  auto chars = chars_in.contiguous();
  auto coff = coff_in.to(chars.device(), at::kLong).contiguous();
  const int64_t K = coff.numel() - 1, HW = H * W, words = (HW + 63) / 64;
  TORCH_CHECK(K >= 0, "rle_decode_bits: offsets need K + 1 entries");
  TORCH_CHECK(HW < (int64_t{1} << 31), "rle_decode_bits: more than 2^31 pixels per mask");
  auto opts = chars.options();
  auto bits = at::empty({K, words}, opts.dtype(at::kLong));
  auto area = at::empty({K}, opts.dtype(at::kDouble));
  if (K == 0) return {bits, area};
  auto bnd = at::empty({std::max<int64_t>(chars.numel(), 1)}, opts.dtype(at::kInt));
  auto nrun = at::empty({K}, opts.dtype(at::kInt));
  hipLaunchKernelGGL(rle_parse_kernel, dim3(static_cast<unsigned>((K + 63) / 64)), 64, 0, stream(), chars.data_ptr<uint8_t>(),
                     coff.data_ptr<int64_t>(), static_cast<int>(K), bnd.data_ptr<int32_t>(), nrun.data_ptr<int32_t>(),
                     area.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  if (words > 0) {
    hipLaunchKernelGGL(rle_fill_kernel, grid_for(K * words, 256, 16384), 256, 0, stream(), bnd.data_ptr<int32_t>(), coff.data_ptr<int64_t>(),
                       nrun.data_ptr<int32_t>(), HW, words, K * words, reinterpret_cast<uint64_t*>(bits.data_ptr<int64_t>()));
    TMX_LAUNCH_CHECK();
  }
  return {bits, area};
}

// ------------------------------------------------------------------------------------------------ batched IoU
constexpr int kIouTile = 16;
constexpr int kIouChunk = 64;

// tiles [T][3] = (image, d0, g0); det rows of image i: det_off[i] .. det_off[i + 1] (same for gt); out block of
// image i at out_off[i], row-major [D_i, G_i]
__global__ void __launch_bounds__(kIouTile * kIouTile) mask_iou_tiles_kernel(
    const uint64_t* __restrict__ dbits, const uint64_t* __restrict__ gbits, const double* __restrict__ darea,
    const double* __restrict__ garea, const bool* __restrict__ crowd, const int64_t* __restrict__ det_off,
    const int64_t* __restrict__ gt_off, const int64_t* __restrict__ out_off, const int32_t* __restrict__ tiles, int64_t W,
    double* __restrict__ out) {
  __shared__ uint64_t sd[kIouTile][kIouChunk + 1];
  __shared__ uint64_t sg[kIouTile][kIouChunk + 1];
  const int img = tiles[3 * blockIdx.x], d0 = tiles[3 * blockIdx.x + 1], g0 = tiles[3 * blockIdx.x + 2];
  const int64_t db = det_off[img], gb = gt_off[img];
  const int D = static_cast<int>(det_off[img + 1] - db), G = static_cast<int>(gt_off[img + 1] - gb);
  const int tid = threadIdx.x;
  const int ld = tid / kIouTile, lg = tid % kIouTile;
  unsigned long long inter = 0;
  for (int64_t w0 = 0; w0 < W; w0 += kIouChunk) {
    for (int e = tid; e < kIouTile * kIouChunk; e += kIouTile * kIouTile) {
      const int r = e / kIouChunk, c = e % kIouChunk;
      const int64_t w = w0 + c;
      sd[r][c] = (d0 + r < D && w < W) ? dbits[(db + d0 + r) * W + w] : 0ull;
      sg[r][c] = (g0 + r < G && w < W) ? gbits[(gb + g0 + r) * W + w] : 0ull;
    }
    __syncthreads();
#pragma unroll 8
    for (int c = 0; c < kIouChunk; ++c) inter += __popcll(sd[ld][c] & sg[lg][c]);
    __syncthreads();
  }
  const int d = d0 + ld, g = g0 + lg;
  if (d >= D || g >= G) return;
  const double i = static_cast<double>(inter);
  const double u = crowd[gb + g] ? darea[db + d] : darea[db + d] + garea[gb + g] - i;
  out[out_off[img] + (int64_t)d * G + g] = u > 0 ? i / u : 0.0;
}

at::Tensor mask_iou_tiles_cuda(const at::Tensor& dbits, const at::Tensor& gbits, const at::Tensor& darea, const at::Tensor& garea,
                               const at::Tensor& crowd, const at::Tensor& det_off, const at::Tensor& gt_off, const at::Tensor& out_off,
                               const at::Tensor& tiles, int64_t total) {
  TORCH_CHECK(dbits.is_cuda() && dbits.scalar_type() == at::kLong && gbits.scalar_type() == at::kLong, "mask_iou_tiles: int64 GPU words");
  TORCH_CHECK(dbits.dim() == 2 && gbits.dim() == 2 && dbits.size(1) == gbits.size(1), "mask_iou_tiles: word count mismatch");
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 3, "mask_iou_tiles: tiles [T, 3]");
  const int64_t I = det_off.numel() - 1;
  TORCH_CHECK(I >= 0 && gt_off.numel() == I + 1 && out_off.numel() >= I, "mask_iou_tiles: offset sizes");
  TORCH_CHECK(darea.numel() == dbits.size(0) && garea.numel() == gbits.size(0) && crowd.numel() == gbits.size(0),
              "mask_iou_tiles: area / crowd sizes");
  const at::DeviceGuard guard(dbits.device());
  auto dev = dbits.device();
  auto out = at::zeros({total}, dbits.options().dtype(at::kDouble));
  const int64_t T = tiles.size(0);
  if (T == 0 || total == 0) return out;
  auto tl = tiles.to(dev, at::kInt).contiguous();
  // the host tile list must stay inside the offsets: validated here (a bad tile would read out of bounds)
  auto doff = det_off.to(at::kLong).contiguous(), goff = gt_off.to(at::kLong).contiguous(), ooff = out_off.to(at::kLong).contiguous();
  {
    auto tc = tiles.to(at::kCPU, at::kInt).contiguous();
    auto dc = doff.cpu(), gc = goff.cpu(), oc = ooff.cpu();
    const int32_t* t = tc.data_ptr<int32_t>();
    const int64_t* dp = dc.data_ptr<int64_t>();
    const int64_t* gp = gc.data_ptr<int64_t>();
    const int64_t* op = oc.data_ptr<int64_t>();
    TORCH_CHECK(dp[I] <= dbits.size(0) && gp[I] <= gbits.size(0), "mask_iou_tiles: offsets exceed the mask rows");
    for (int64_t i = 0; i < T; ++i) {
      const int img = t[3 * i], d0 = t[3 * i + 1], g0 = t[3 * i + 2];
      TORCH_CHECK(img >= 0 && img < I && d0 >= 0 && g0 >= 0 && d0 < dp[img + 1] - dp[img] && g0 < gp[img + 1] - gp[img],
                  "mask_iou_tiles: tile out of range");
      TORCH_CHECK(op[img] + (dp[img + 1] - dp[img]) * (gp[img + 1] - gp[img]) <= total, "mask_iou_tiles: output block out of range");
    }
  }
  auto db = dbits.contiguous(), gb = gbits.contiguous();
  auto da = darea.to(dev, at::kDouble).contiguous(), ga = garea.to(dev, at::kDouble).contiguous();
  auto cr = crowd.to(dev, at::kBool).contiguous();
  auto dd = doff.to(dev), gd = goff.to(dev), od = ooff.to(dev);
  hipLaunchKernelGGL(mask_iou_tiles_kernel, dim3(static_cast<unsigned>(T)), kIouTile * kIouTile, 0, stream(),
                     reinterpret_cast<const uint64_t*>(db.data_ptr<int64_t>()), reinterpret_cast<const uint64_t*>(gb.data_ptr<int64_t>()),
                     da.data_ptr<double>(), ga.data_ptr<double>(), cr.data_ptr<bool>(), dd.data_ptr<int64_t>(), gd.data_ptr<int64_t>(),
                     od.data_ptr<int64_t>(), tl.data_ptr<int32_t>(), dbits.size(1), out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

// ------------------------------------------------------------------------------------------------------- CPU
static void counts_to_chars(const std::vector<int64_t>& cnts, std::vector<uint8_t>& s) {
  for (size_t i = 0; i < cnts.size(); ++i) {
    long long x = cnts[i];
    if (i > 2) x -= cnts[i - 2];
    bool more = true;
    while (more) {
      int c = static_cast<int>(x & 0x1f);
      x >>= 5;
      more = (c & 0x10) ? x != -1 : x != 0;
      if (more) c |= 0x20;
      s.push_back(static_cast<uint8_t>(c + 48));
    }
  }
}

std::tuple<at::Tensor, at::Tensor> rle_encode_cpu(const at::Tensor& masks_in) {
  TORCH_CHECK(masks_in.dim() == 3, "rle_encode: expected [K, H, W] masks");
  auto masks = masks_in.ne(0).to(at::kByte).contiguous();
  const int64_t K = masks.size(0), H = masks.size(1), W = masks.size(2);
  const uint8_t* m = masks.data_ptr<uint8_t>();
  std::vector<std::vector<uint8_t>> strs(K);
  at::parallel_for(0, K, 1, [&](int64_t b, int64_t e) {
    std::vector<int64_t> cnts;
    for (int64_t k = b; k < e; ++k) {
      cnts.clear();
      const uint8_t* mk = m + k * H * W;
      uint8_t p = 0;
      int64_t c = 0;
      for (int64_t x = 0; x < W; ++x)
        for (int64_t y = 0; y < H; ++y) {
          const uint8_t v = mk[y * W + x];
          if (v != p) {
            cnts.push_back(c);
            c = 0;
            p = v;
          }
          ++c;
        }
      cnts.push_back(c);
      counts_to_chars(cnts, strs[k]);
    }
  });
  auto off = at::empty({K + 1}, at::TensorOptions().dtype(at::kLong));
  int64_t* o = off.data_ptr<int64_t>();
  o[0] = 0;
  for (int64_t k = 0; k < K; ++k) o[k + 1] = o[k] + static_cast<int64_t>(strs[k].size());
  auto chars = at::empty({o[K]}, at::TensorOptions().dtype(at::kByte));
  uint8_t* cp = chars.data_ptr<uint8_t>();
  for (int64_t k = 0; k < K; ++k) std::copy(strs[k].begin(), strs[k].end(), cp + o[k]);
  return {chars, off};
}

static void parse_counts(const uint8_t* s, int64_t len, std::vector<int64_t>& cnts) {
  cnts.clear();
  int64_t p = 0;
  while (p < len) {
    long long x = 0;
    int sh = 0;
    bool more = true;
    while (more && p < len) {
      const int c = static_cast<int>(s[p++]) - 48;
      x |= static_cast<long long>(c & 0x1f) << sh;
      more = (c & 0x20) != 0;
      sh += 5;
      if (!more && (c & 0x10)) x |= -1ll << sh;
    }
    if (cnts.size() > 2) x += cnts[cnts.size() - 2];
    cnts.push_back(x);
  }
}

std::tuple<at::Tensor, at::Tensor> rle_decode_bits_cpu(const at::Tensor& chars_in, const at::Tensor& coff_in, int64_t H, int64_t W) {
  auto chars = chars_in.contiguous();
  auto coff = coff_in.to(at::kLong).contiguous();
  const int64_t K = coff.numel() - 1, HW = H * W, words = (HW + 63) / 64;
  auto bits = at::zeros({K, words}, at::TensorOptions().dtype(at::kLong));
  auto area = at::zeros({K}, at::TensorOptions().dtype(at::kDouble));
  const uint8_t* cs = chars.data_ptr<uint8_t>();
  const int64_t* co = coff.data_ptr<int64_t>();
  uint64_t* bp = reinterpret_cast<uint64_t*>(bits.data_ptr<int64_t>());
  double* ap = area.data_ptr<double>();
  at::parallel_for(0, K, 1, [&](int64_t b, int64_t e) {
    std::vector<int64_t> cnts;
    for (int64_t k = b; k < e; ++k) {
      parse_counts(cs + co[k], co[k + 1] - co[k], cnts);
      int64_t pos = 0, fg = 0;
      uint64_t* row = bp + k * words;
      for (size_t j = 0; j < cnts.size(); ++j) {
        const int64_t s0 = pos, e0 = std::min<int64_t>(pos + cnts[j], HW);
        if ((j & 1) && e0 > s0) {
          fg += cnts[j];
          for (int64_t q = s0; q < e0; ++q) row[q >> 6] |= uint64_t{1} << (q & 63);
        }
        pos += cnts[j];
      }
      ap[k] = static_cast<double>(fg);
    }
  });
  return {bits, area};
}

at::Tensor mask_iou_tiles_cpu(const at::Tensor& dbits_in, const at::Tensor& gbits_in, const at::Tensor& darea_in, const at::Tensor& garea_in,
                              const at::Tensor& crowd_in, const at::Tensor& det_off_in, const at::Tensor& gt_off_in, const at::Tensor& out_off_in,
                              const at::Tensor& tiles, int64_t total) {
  auto dbits = dbits_in.contiguous(), gbits = gbits_in.contiguous();
  auto darea = darea_in.to(at::kDouble).contiguous(), garea = garea_in.to(at::kDouble).contiguous();
  auto crowd = crowd_in.to(at::kBool).contiguous();
  auto doff = det_off_in.to(at::kLong).contiguous(), goff = gt_off_in.to(at::kLong).contiguous(), ooff = out_off_in.to(at::kLong).contiguous();
  auto out = at::zeros({total}, at::TensorOptions().dtype(at::kDouble));
  const int64_t I = doff.numel() - 1, W = dbits.size(1);
  const uint64_t* db = reinterpret_cast<const uint64_t*>(dbits.data_ptr<int64_t>());
  const uint64_t* gbp = reinterpret_cast<const uint64_t*>(gbits.data_ptr<int64_t>());
  const double* da = darea.data_ptr<double>();
  const double* ga = garea.data_ptr<double>();
  const bool* cr = crowd.data_ptr<bool>();
  const int64_t* dp = doff.data_ptr<int64_t>();
  const int64_t* gp = goff.data_ptr<int64_t>();
  const int64_t* op = ooff.data_ptr<int64_t>();
  double* o = out.data_ptr<double>();
  at::parallel_for(0, I, 1, [&](int64_t b, int64_t e) {
    for (int64_t img = b; img < e; ++img) {
      const int64_t D = dp[img + 1] - dp[img], G = gp[img + 1] - gp[img];
      for (int64_t d = 0; d < D; ++d)
        for (int64_t g = 0; g < G; ++g) {
          const uint64_t* a = db + (dp[img] + d) * W;
          const uint64_t* c = gbp + (gp[img] + g) * W;
          uint64_t inter = 0;
          for (int64_t w = 0; w < W; ++w) inter += static_cast<uint64_t>(__builtin_popcountll(a[w] & c[w]));
          const double i = static_cast<double>(inter);
          const double u = cr[gp[img] + g] ? da[dp[img] + d] : da[dp[img] + d] + ga[gp[img] + g] - i;
          o[op[img] + d * G + g] = u > 0 ? i / u : 0.0;
        }
    }
  });
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("rle_encode(Tensor masks) -> (Tensor, Tensor)");
  m.def("rle_decode_bits(Tensor chars, Tensor offsets, int H, int W) -> (Tensor, Tensor)");
  m.def("mask_iou_tiles(Tensor det_bits, Tensor gt_bits, Tensor det_area, Tensor gt_area, Tensor gt_crowd, Tensor det_off, "
        "Tensor gt_off, Tensor out_off, Tensor tiles, int total) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("rle_encode", &tmx::rle_encode_cuda);
  m.impl("rle_decode_bits", &tmx::rle_decode_bits_cuda);
  m.impl("mask_iou_tiles", &tmx::mask_iou_tiles_cuda);
}

TORCH_LIBRARY_IMPL(tmx, CPU, m) {
  m.impl("rle_encode", &tmx::rle_encode_cpu);
  m.impl("rle_decode_bits", &tmx::rle_decode_bits_cpu);
  m.impl("mask_iou_tiles", &tmx::mask_iou_tiles_cpu);
}
