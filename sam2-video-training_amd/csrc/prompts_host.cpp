// Host half of the per-clip prompt stage, native (reference sam2_video/utils/masks.py:13-50 and
// prompts.py:13-97, called from sam2model.py:181-236 once per training step on frame 0).
//
// The reference runs cv2 on the CPU: a 5x5-ellipse opening of every category mask, 8-connected
// components in raster order (one object per component), then one click per object (centre of
// mass) or its bounding box.  It is CPU work on the training thread every step, so its cost adds
// to the step unless it is shorter than the GPU's: this file does it in a few passes of byte
// vectors per category (one thread per category) instead of per-object full-image scans.
//
// Opening.  cv2's 5x5 ellipse (rows 0 and 4 hold only the centre pixel, rows 1-3 are full) is the
// union of a 5-wide x 3-tall rectangle and a 1-wide x 5-tall bar, so erosion by it is the AND of
// a separable rectangle erosion and a vertical bar erosion, and dilation the OR of the two
// dilations.  Borders follow the reference: erosion treats outside pixels as
// set, dilation as clear.
//
// Labelling.  Two-pass union-find over the 8-neighbourhood (W, NW, N, NE); each set's root is
// its smallest provisional label, provisional labels are created in raster order, so numbering
// roots by increasing label numbers components by their first pixel in raster order (the order
// cv2.connectedComponents / scipy.ndimage.label give).
//
// Moments.  Per object: pixel count, sum of y, sum of x (exact int64), y/x extremes.  The centre
// of mass is sum / count in double, exactly what the reference's float64 reduction of integer
// products gives.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kStats = 7;  // count, sum_y, sum_x, y_min, y_max, x_min, x_max

// o[y][x] = op over a[y][x-R .. x+R]; pixels outside the row count as `border`
template <int R, bool AND>
void hpass(const uint8_t* a, uint8_t* o, int H, int W, uint8_t border) {
  auto op = [](uint8_t u, uint8_t v) -> uint8_t { return AND ? (uint8_t)(u & v) : (uint8_t)(u | v); };
  auto edge = [&](const uint8_t* s, int x) {
    uint8_t v = AND ? 1 : 0;
    for (int k = -R; k <= R; ++k) v = op(v, (x + k < 0 || x + k >= W) ? border : s[x + k]);
    return v;
  };
  for (int y = 0; y < H; ++y) {
    const uint8_t* s = a + (int64_t)y * W;
    uint8_t* d = o + (int64_t)y * W;
    const int lo = std::min(R, W), hi = std::max(lo, W - R);
    for (int x = 0; x < lo; ++x) d[x] = edge(s, x);
    for (int x = lo; x < hi; ++x) {  // fixed-width window: vectorised
      uint8_t v = s[x];
      for (int k = 1; k <= R; ++k) v = op(v, op(s[x - k], s[x + k]));
      d[x] = v;
    }
    for (int x = hi; x < W; ++x) d[x] = edge(s, x);
  }
}

// o[y][x] = op over a[y-R .. y+R][x]; rows outside the image count as `border`
template <int R, bool AND>
void vpass(const uint8_t* a, uint8_t* o, int H, int W, uint8_t border) {
  for (int y = 0; y < H; ++y) {
    uint8_t* d = o + (int64_t)y * W;
    std::memset(d, AND ? 1 : 0, W);
    for (int k = -R; k <= R; ++k) {
      const int yy = y + k;
      if (yy < 0 || yy >= H) {
        if (AND && !border) { std::memset(d, 0, W); break; }
        if (!AND && border) { std::memset(d, 1, W); break; }
        continue;
      }
      const uint8_t* s = a + (int64_t)yy * W;
      if (AND)
        for (int x = 0; x < W; ++x) d[x] &= s[x];
      else
        for (int x = 0; x < W; ++x) d[x] |= s[x];
    }
  }
}

// 5x5-ellipse opening of a 0/1 mask (masks.py:19-22); t0..t2 are H*W scratch.  The `H` rows may be
// a window of the image when every row outside it is clear and two clear rows separate each window
// edge that is not the image's own from the nearest set pixel: the erosion is then 0 on those
// padding rows whatever the border says, and the dilation of the eroded rows stays inside.
void open_ellipse5(const uint8_t* m, uint8_t* out, uint8_t* t0, uint8_t* t1, uint8_t* t2, int H, int W) {
  const int64_t n = (int64_t)H * W;
  hpass<2, true>(m, t0, H, W, 1);   // erode: 5 wide ...
  vpass<1, true>(t0, t1, H, W, 1);  //        ... x 3 tall
  vpass<2, true>(m, t2, H, W, 1);   //        1 wide x 5 tall
  for (int64_t i = 0; i < n; ++i) t1[i] &= t2[i];  // eroded
  hpass<2, false>(t1, t0, H, W, 0);  // dilate: 5 x 3
  vpass<1, false>(t0, out, H, W, 0);
  vpass<2, false>(t1, t2, H, W, 0);  //         1 x 5
  for (int64_t i = 0; i < n; ++i) out[i] |= t2[i];
}

struct Run {
  int y, x0, x1;  // [x0, x1) of row y
};

int find_root(std::vector<int32_t>& par, int32_t a) {
  while (par[a] != a) {
    par[a] = par[par[a]];
    a = par[a];
  }
  return a;
}

// 8-connected labelling of a 0/1 mask by runs: runs of each row are united with the runs of the
// row above they touch (overlap or diagonal contact); runs are numbered in raster order and each
// set's root is its smallest run, so numbering roots in order numbers components by their first
// pixel in raster order.  Appends the components' moments to `stats`; when `lab` is given writes
// lab[y][x] = label_base + component index (1-based) on the runs (the caller clears the rest).
int label8(const uint8_t* m, int H, int W, int y_off, int32_t* lab, int32_t label_base, std::vector<Run>& runs,
           std::vector<int32_t>& par, std::vector<int64_t>& stats) {
  runs.clear();
  par.clear();
  size_t prev_lo = 0, prev_hi = 0;  // runs of the previous row
  for (int y = 0; y < H; ++y) {
    const uint8_t* row = m + (int64_t)y * W;
    const size_t cur_lo = runs.size();
    const uint8_t* p = row;
    const uint8_t* end = row + W;
    while (p < end) {
      const uint8_t* q = (const uint8_t*)std::memchr(p, 1, end - p);
      if (!q) break;
      const uint8_t* r = (const uint8_t*)std::memchr(q, 0, end - q);
      if (!r) r = end;
      runs.push_back({y, (int)(q - row), (int)(r - row)});
      par.push_back((int32_t)par.size());
      p = r;
    }
    const size_t cur_hi = runs.size();
    if (y > 0 && prev_hi > prev_lo) {
      size_t j = prev_lo;
      for (size_t i = cur_lo; i < cur_hi; ++i) {
        const Run& c = runs[i];
        while (j < prev_hi && runs[j].x1 < c.x0) ++j;  // ends left of c's diagonal reach
        for (size_t k = j; k < prev_hi && runs[k].x0 <= c.x1; ++k) {
          int32_t a = find_root(par, (int32_t)i), b = find_root(par, (int32_t)k);
          if (a < b) par[b] = a;
          else if (b < a) par[a] = b;
        }
      }
    }
    prev_lo = cur_lo;
    prev_hi = cur_hi;
  }
  const int32_t nr = (int32_t)runs.size();
  std::vector<int32_t> id(nr, 0);
  int n = 0;
  for (int32_t k = 0; k < nr; ++k)
    id[k] = (find_root(par, k) == k) ? ++n : id[find_root(par, k)];  // roots precede their runs
  const size_t base = stats.size();
  stats.resize(base + (size_t)n * kStats);
  for (int i = 0; i < n; ++i) {
    int64_t* s = &stats[base + (size_t)i * kStats];
    s[0] = s[1] = s[2] = 0;
    s[3] = INT64_MAX; s[4] = -1; s[5] = INT64_MAX; s[6] = -1;
  }
  for (int32_t k = 0; k < nr; ++k) {
    const Run& r = runs[k];
    const int64_t len = r.x1 - r.x0, y = r.y + y_off;
    int64_t* s = &stats[base + (size_t)(id[k] - 1) * kStats];
    s[0] += len;
    s[1] += y * len;
    s[2] += (int64_t)(r.x0 + r.x1 - 1) * len / 2;
    s[3] = std::min<int64_t>(s[3], y); s[4] = std::max<int64_t>(s[4], y);
    s[5] = std::min<int64_t>(s[5], r.x0); s[6] = std::max<int64_t>(s[6], r.x1 - 1);
    if (lab) {
      int32_t* l = lab + (int64_t)r.y * W;
      for (int x = r.x0; x < r.x1; ++x) l[x] = label_base + id[k];
    }
  }
  return n;
}

template <class F>
void parallel_for(int n, int threads, F&& fn) {
  threads = std::max(1, std::min(threads, n));
  if (threads == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (int i = t; i < n; i += threads) fn(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

// cat_to_obj_mask (masks.py:31-50) + find_connected_components (masks.py:13-28) over N category
// masks [N, H, W] (0/1 bytes).  Objects are numbered category-major, raster order within a
// category.  On success (0): *n_obj objects, obj_cat[o] its category, stats[o*7 ..] its moments
// (count, sum_y, sum_x, y_min, y_max, x_min, x_max), and when `lab` is given lab[c][y][x] = 1 +
// the global object index (0 = background).  Returns 2 with *n_obj = the count needed when more
// than max_obj objects exist (obj_cat / stats untouched, `lab` unspecified), 1 on bad arguments.
int s2h_prompt_objects(int N, int H, int W, const uint8_t* masks, int max_obj, int* n_obj, int32_t* obj_cat,
                       int64_t* stats, int32_t* lab, int threads) {
  if (N < 0 || H <= 0 || W <= 0 || !masks || !n_obj || max_obj < 0 || (max_obj && (!obj_cat || !stats)))
    return 1;
  const int64_t hw = (int64_t)H * W;
  std::vector<std::vector<int64_t>> cst(N);
  std::vector<int> cnt(N, 0);
  if (lab) std::memset(lab, 0, (size_t)N * hw * sizeof(int32_t));
  parallel_for(N, threads, [&](int c) {
    const uint8_t* m = masks + c * hw;
    // rows holding set pixels; the opening only shrinks, so it is computed on those rows plus two
    // clear rows either side (where the image has them), which is exact (see open_ellipse5)
    int y0 = H, y1 = -1;
    for (int y = 0; y < H; ++y) {
      const uint8_t* row = m + (int64_t)y * W;
      uint8_t any = 0;
      for (int x = 0; x < W; ++x) any |= row[x];
      if (any) {
        y0 = std::min(y0, y);
        y1 = y;
      }
    }
    if (y1 < 0) return;  // masks.py:41: an empty category contributes no object
    const int a = std::max(0, y0 - 2), b = std::min(H, y1 + 3), h = b - a;
    const int64_t n = (int64_t)h * W;
    std::vector<uint8_t> buf((size_t)n * 5);
    uint8_t* bin = buf.data();
    const uint8_t* src = m + (int64_t)a * W;
    for (int64_t i = 0; i < n; ++i) bin[i] = src[i] != 0;
    open_ellipse5(bin, bin + n, bin + 2 * n, bin + 3 * n, bin + 4 * n, h, W);
    std::vector<Run> runs;
    std::vector<int32_t> par;
    cnt[c] = label8(bin + n, h, W, a, lab ? lab + c * hw + (int64_t)a * W : nullptr, 0, runs, par, cst[c]);
  });
  int total = 0;
  for (int c = 0; c < N; ++c) total += cnt[c];
  *n_obj = total;
  if (total > max_obj) return 2;
  int base = 0;
  for (int c = 0; c < N; ++c) {
    for (int i = 0; i < cnt[c]; ++i) obj_cat[base + i] = c;
    if (cnt[c])  // an empty category's vector may have no storage (memcpy from null is UB even for 0 bytes)
      std::memcpy(stats + (int64_t)base * kStats, cst[c].data(), (size_t)cnt[c] * kStats * sizeof(int64_t));
    if (lab && base) {
      int32_t* l = lab + c * hw;
      for (int64_t i = 0; i < hw; ++i)
        if (l[i]) l[i] += base;
    }
    base += cnt[c];
  }
  return 0;
}

// object masks from s2h_prompt_objects' labels: out[o][y][x] = 1.0f where object o is, else 0
// (the float [O, H, W] masks cat_to_obj_mask returns)
int s2h_prompt_object_masks(int N, int H, int W, const int32_t* lab, int n_obj, float* out, int threads) {
  if (N < 0 || H <= 0 || W <= 0 || n_obj < 0 || (n_obj && (!lab || !out))) return 1;
  const int64_t hw = (int64_t)H * W;
  if (n_obj) std::memset(out, 0, (size_t)n_obj * hw * sizeof(float));
  parallel_for(N, threads, [&](int c) {
    const int32_t* l = lab + c * hw;
    for (int64_t i = 0; i < hw; ++i) {
      const int32_t o = l[i];
      if (o > 0 && o <= n_obj) out[(int64_t)(o - 1) * hw + i] = 1.0f;
    }
  });
  return 0;
}

// moments of B masks [B, H, W] (0/1 bytes) taken whole, no opening: stats[b*7 ..] as above
// (generate_point_prompt's centre of mass, prompts.py:36-44; generate_box_prompt's corners,
// prompts.py:86-95)
int s2h_mask_moments(int B, int H, int W, const uint8_t* masks, int64_t* stats, int threads) {
  if (B < 0 || H <= 0 || W <= 0 || (B && (!masks || !stats))) return 1;
  const int64_t hw = (int64_t)H * W;
  parallel_for(B, threads, [&](int b) {
    const uint8_t* m = masks + b * hw;
    int64_t cnt = 0, sy = 0, sx = 0, y0 = H, y1 = -1, x0 = W, x1 = -1;
    for (int y = 0; y < H; ++y) {
      const uint8_t* row = m + (int64_t)y * W;
      int64_t rc = 0, rs = 0;
      int first = -1, last = -1;
      for (int x = 0; x < W; ++x)
        if (row[x]) {
          rc += 1;
          rs += x;
          if (first < 0) first = x;
          last = x;
        }
      if (!rc) continue;
      cnt += rc; sy += rc * y; sx += rs;
      y0 = std::min<int64_t>(y0, y); y1 = y;
      x0 = std::min<int64_t>(x0, first); x1 = std::max<int64_t>(x1, last);
    }
    int64_t* s = stats + (int64_t)b * kStats;
    s[0] = cnt; s[1] = sy; s[2] = sx; s[3] = y0; s[4] = y1; s[5] = x0; s[6] = x1;
  });
  return 0;
}

}  // extern "C"
