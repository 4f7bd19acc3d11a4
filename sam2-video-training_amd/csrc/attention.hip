// Flash attention forward + backward for every attention on the SAM2 step:
//   * Hiera windowed / q-pooled / global MHSA   (hieradet.py:56-81)      head_dim 56/96/72
//   * memory-attention RoPE self + cross attn   (transformer.py:275-311) head_dim 256, Lk <= 7*1028
//   * two-way decoder token<->image attention   (transformer.py:231-248) head_dim 32 / 16
// Softmax(scale * Q K^T) V with online (base-2) softmax, optional in-kernel
// dropout on P (counter-hash mask, regenerated in backward), LSE saved for the
// backward.  Q/K/V/O are addressed with (batch, head, row) strides and a
// contiguous head dim, so the projections' [B, L, H, d] outputs are consumed in
// place.  head_dim is zero-padded to DP (multiple of 32) in registers/LDS only.
//
// Backward = two kernels (no atomics): dQ per query block, dK/dV per key block.
#include "common.h"

struct AttnArgs {
  int B, H, Lq, Lk, D;
  const void* q; int64_t sqb, sqh, sql;
  const void* k; int64_t skb, skh, skl;
  const void* v; int64_t svb, svh, svl;
  void* o; int64_t sob, soh, sol;        // forward: O ; backward: dO
  const void* fo; int64_t sfb, sfh, sfl; // backward: forward output O (for Di)
  void* dq; int64_t sdqb, sdqh, sdql;
  void* dk; int64_t sdkb, sdkh, sdkl;
  void* dv; int64_t sdvb, sdvh, sdvl;
  float* lse;  // [B*H*Lq]
  float* di;   // [B*H*Lq] backward workspace: rowsum(dO*O)
  float scale;
  float p_drop;
  uint64_t seed;
  const uint64_t* seed_off;
  uint64_t idx0;  // dropout element-index offset (frame slot of a frame-stacked batch)
};

int s2h_prof_begin(hipStream_t st, int kind, int64_t m0, int64_t m1, int64_t m2, int64_t m3, int64_t m4);
void s2h_prof_end(int slot, hipStream_t st);
// flash.hip (bf16 long-sequence forward)
int s2h_flash_eligible(int dt, int Lq, int D);
int64_t s2h_flash_ws_bytes(int B, int H, int Lq, int Lk, int D);
int s2h_flash_fwd(int B, int H, int Lq, int Lk, int D, const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                  const void* k, int64_t skb, int64_t skh, int64_t skl, const void* v, int64_t svb, int64_t svh,
                  int64_t svl, void* o, int64_t sob, int64_t soh, int64_t sol, float* lse, float scale, float p_drop,
                  uint64_t seed, uint64_t idx0, uint32_t* keep, void* ws, int64_t ws_bytes, hipStream_t st);

int s2h_flash_bwd_eligible(int dt, int Lq, int D);
int64_t s2h_flash_bwd_ws_bytes(int B, int H, int Lq, int Lk, int D);
int s2h_flash_bwd(int B, int H, int Lq, int Lk, int D, const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                  const void* k, int64_t skb, int64_t skh, int64_t skl, const void* v, int64_t svb, int64_t svh,
                  int64_t svl, const void* o, int64_t sob, int64_t soh, int64_t sol, const void* dout, int64_t sgb,
                  int64_t sgh, int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql, void* dk, int64_t sdkb,
                  int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvb, int64_t sdvh, int64_t sdvl, const float* lse,
                  float* di_ws, float scale, float p_drop, uint64_t seed, uint64_t idx0, const uint32_t* keep, void* ws,
                  int64_t ws_bytes, hipStream_t st);

// 32-bit words of the dropout keep bitmap of one attention launch (flash path, head_dim 256):
// B*H*Lq rows of 2 * ceil(Lk / 64) words.
extern "C" int64_t s2h_attn_keep_words(int B, int H, int Lq, int Lk) {
  return (int64_t)B * H * Lq * 2 * ((Lk + 63) / 64);
}

// Workspace the backward wants (key-split dQ partials of the flash path); 0 = none.
extern "C" int64_t s2h_attn_bwd_ws_bytes(int dt, int B, int H, int Lq, int Lk, int D) {
  return s2h_flash_bwd_eligible(dt, Lq, D) ? s2h_flash_bwd_ws_bytes(B, H, Lq, Lk, D) : 0;
}

// Workspace the forward wants (key-split partials of the flash path); 0 = none.
extern "C" int64_t s2h_attn_fwd_ws_bytes(int dt, int B, int H, int Lq, int Lk, int D) {
  return s2h_flash_eligible(dt, Lq, D) ? s2h_flash_ws_bytes(B, H, Lq, Lk, D) : 0;
}

#define LOG2E 1.4426950408889634f
#define LN2 0.6931471805599453f

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16> { static constexpr int BKEY = 64, NW_DKV = 4; };
template <> struct AttnCfg<float> { static constexpr int BKEY = 32, NW_DKV = 2; };
template <typename T, int DP> struct DkvBQ {
  static constexpr int v = DP >= 256 ? (sizeof(T) == 2 ? 32 : 16) : (sizeof(T) == 2 ? 64 : 32);
};

// Load ROWS x DP tile (rows r0.., d contiguous) into LDS, natural [row][d] layout.
template <typename T, int ROWS, int DP, int STRIDE, int NTHR>
__device__ __forceinline__ void lds_load_rows(T* dst, const T* src, int64_t ld, int r0, int nrows, int D, int tid) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NV = ROWS * DP / VEC;
  for (int v = tid; v < NV; v += NTHR) {
    int row = v / (DP / VEC), d = (v % (DP / VEC)) * VEC;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (r0 + row < nrows && d < D) val = *(const uint4*)(src + (int64_t)(r0 + row) * ld + d);
    *(uint4*)(dst + row * STRIDE + d) = val;
  }
}
// Same source tile stored transposed: dst[d][row].
template <typename T, int ROWS, int DP, int STRIDE, int NTHR>
__device__ __forceinline__ void lds_load_rows_t(T* dst, const T* src, int64_t ld, int r0, int nrows, int D, int tid) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NV = ROWS * DP / VEC;
  for (int v = tid; v < NV; v += NTHR) {
    int row = v % ROWS, d = (v / ROWS) * VEC;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (r0 + row < nrows && d < D) val = *(const uint4*)(src + (int64_t)(r0 + row) * ld + d);
    const T* t = (const T*)&val;
#pragma unroll
    for (int j = 0; j < VEC; ++j) dst[(d + j) * STRIDE + row] = t[j];
  }
}
// A-operand fragment of 16 rows x KSTEP straight from global (rows >= nrows, d >= D -> 0)
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag frag_global(const T* base, int64_t ld, int row, int nrows, int d, int D) {
  using MF = Mfma<T>;
  if (row < nrows && d < D) {
    if constexpr (sizeof(T) == 2) return *(const bf16x8*)(base + (int64_t)row * ld + d);
    else return base[(int64_t)row * ld + d];
  }
  return MF::zero();
}

// bf16 B-operand fragment (k = k0 .. k0+31, n = n0 .. n0+15) read from a NATURAL [k][n] LDS
// image with transposing LDS reads (ds_read_b64_tr_b16, two per fragment): replaces the
// transposed tile copies (lds_load_rows_t: eight 2-byte LDS stores per 16-B vector) of V in the
// forward, K in dQ and Q / dO in dK / dV.  ld (elements) and n0 keep every read 8-B aligned.
typedef short attn_v4i16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 tr_bfrag(const bf16* img, int ld, int k0, int n0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16* a0 = img + (k0 + 8 * g + q) * ld + n0 + 4 * p;
  const bf16* a1 = a0 + 4 * ld;
  typedef __attribute__((address_space(3))) attn_v4i16 lds_v4;
  const attn_v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a0);
  const attn_v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a1);
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}
template <typename T> __device__ __forceinline__ typename Mfma<T>::frag tr_or_load(const T* nat, int ldn, const T* tr, int ldt,
                                                                                    int k0, int n0, int lane) {
  // B operand B[k][n] for k = k0 + 8(lane >> 4) + j, n = n0 + (lane & 15): bf16 from the natural
  // image, fp32 from the transposed copy (one element per lane)
  if constexpr (sizeof(T) == 2) return tr_bfrag(nat, ldn, k0, n0, lane);
  else return Mfma<T>::load(&tr[(n0 + (lane & 15)) * ldt + k0 + (lane >> 4) * Mfma<T>::KPL]);
}

// ------------------------------------------------------------------ forward
template <typename T, int DP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int BKEY = AttnCfg<T>::BKEY;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int KS = DP + VEC, VS = BKEY + VEC, PS = BKEY + VEC;
  constexpr int NQF = DP / MF::KSTEP, NB = BKEY / 16, ND = DP / 16;
  constexpr bool TRR = sizeof(T) == 2;  // bf16: V natural, read transposed
  constexpr int VBUF = TRR ? BKEY * KS : DP * VS;
  __shared__ __attribute__((aligned(16))) T smem[BKEY * KS + VBUF + 4 * 16 * PS];
  T* Ks = smem;
  T* Vt = Ks + BKEY * KS;  // [key][d] (bf16) or [d][key] (fp32)
  T* Ps = Vt + VBUF;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int qw = blockIdx.x * 64 + w * 16;  // first query row of this wave
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  typename MF::frag qf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s)
    qf[s] = frag_global<T>(Q, a.sql, qw + (lane & 15), a.Lq, s * MF::KSTEP + (lane >> 4) * MF::KPL, a.D);

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -INFINITY; l[r] = 0.f; }

  const int nkt = (a.Lk + BKEY - 1) / BKEY;
  T* Pw = Ps + w * 16 * PS;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKEY;
    __syncthreads();
    lds_load_rows<T, BKEY, DP, KS, 256>(Ks, K, a.skl, k0, a.Lk, a.D, tid);
    if constexpr (TRR) lds_load_rows<T, BKEY, DP, KS, 256>(Vt, V, a.svl, k0, a.Lk, a.D, tid);
    else lds_load_rows_t<T, BKEY, DP, VS, 256>(Vt, V, a.svl, k0, a.Lk, a.D, tid);
    __syncthreads();

    f32x4 s[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NQF; ++t) {
        typename MF::frag bk = MF::load(&Ks[(j * 16 + (lane & 15)) * KS + t * MF::KSTEP + (lane >> 4) * MF::KPL]);
        s[j] = MF::mma(qf[t], bk, s[j]);
      }
    }
    float mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const bool kvalid = k0 + j * 16 + (lane & 15) < a.Lk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = kvalid ? s[j][r] * sl2 : -INFINITY;
        s[j][r] = x;
        mx[r] = fmaxf(mx[r], x);
      }
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mx[r] = row16_max(mx[r]);
      float mn = fmaxf(m[r], mx[r]);
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
      rs[r] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int key = k0 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = exp2f(s[j][r] - m[r]);
        rs[r] += p;
        if (drop) {
          const int qi = qw + (lane >> 4) * 4 + r;
          uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qi) * (uint64_t)a.Lk + key;
          p = s2h_keep(a.seed, idx, thresh) ? p * inv_keep : 0.f;
        }
        Pw[((lane >> 4) * 4 + r) * PS + j * 16 + (lane & 15)] = from_f32<T>(p);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) l[r] = l[r] * alpha[r] + row16_sum(rs[r]);
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[d][r] *= alpha[r];
    __syncthreads();
    constexpr int NPF = BKEY / MF::KSTEP;
    typename MF::frag pf[NPF];
#pragma unroll
    for (int t = 0; t < NPF; ++t) pf[t] = MF::load(&Pw[(lane & 15) * PS + t * MF::KSTEP + (lane >> 4) * MF::KPL]);
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int t = 0; t < NPF; ++t) {
        typename MF::frag bv = tr_or_load<T>(Vt, KS, Vt, VS, t * MF::KSTEP, d * 16, lane);
        o[d] = MF::mma(pf[t], bv, o[d]);
      }
  }

  T* O = (T*)a.o + b * a.sob + h * a.soh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = qw + (lane >> 4) * 4 + r;
    const float inv = 1.f / l[r];
    if (row < a.Lq) {
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int col = d * 16 + (lane & 15);
        if (col < a.D) O[(int64_t)row * a.sol + col] = from_f32<T>(o[d][r] * inv);
      }
      if ((lane & 15) == 0) a.lse[(int64_t)bh * a.Lq + row] = (m[r] + log2f(l[r])) * LN2;
    }
  }
}

// ------------------------------------------------- backward: Di = rowsum(dO*O)
// 2^lpr_log2 lanes per row (the fewest that cover D with 16-B vectors when `vec`), so short head
// dims (the decoder's 16 over 852k rows) do not launch one wave per row
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(AttnArgs a, int lpr_log2, int vec) {
  constexpr int V = 16 / sizeof(T);
  const int lpr = 1 << lpr_log2;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> lpr_log2;
  const int sub = threadIdx.x & (lpr - 1);
  const int64_t nrows = (int64_t)a.B * a.H * a.Lq;
  float acc = 0.f;
  if (row < nrows) {
    const int qi = row % a.Lq;
    const int bh = row / a.Lq, b = bh / a.H, h = bh % a.H;
    const T* dO = (const T*)a.o + b * a.sob + h * a.soh + (int64_t)qi * a.sol;
    const T* O = (const T*)a.fo + b * a.sfb + h * a.sfh + (int64_t)qi * a.sfl;
    if (vec) {
      for (int d = sub * V; d < a.D; d += lpr * V) {
        const uint4 gu = *(const uint4*)(dO + d), ou = *(const uint4*)(O + d);
        const T* gb = (const T*)&gu;
        const T* ob = (const T*)&ou;
#pragma unroll
        for (int e = 0; e < V; ++e) acc += to_f32(gb[e]) * to_f32(ob[e]);
      }
    } else {
      for (int d = sub; d < a.D; d += lpr) acc += to_f32(dO[d]) * to_f32(O[d]);
    }
  }
  for (int off = lpr >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (row < nrows && sub == 0) a.di[row] = acc;
}

// ------------------------------------------------------- backward: dQ
template <typename T, int DP>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int BKEY = AttnCfg<T>::BKEY;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int KS = DP + VEC, TS = BKEY + VEC, PS = BKEY + VEC;
  constexpr int NQF = DP / MF::KSTEP, NB = BKEY / 16, ND = DP / 16;
  constexpr bool TRR = sizeof(T) == 2;  // bf16: K^T fragments by transposing reads of Ks
  constexpr int KTBUF = TRR ? 0 : DP * TS;
  __shared__ __attribute__((aligned(16))) T smem[2 * BKEY * KS + KTBUF + 4 * 16 * PS];
  T* Ks = smem;
  T* Vs = Ks + BKEY * KS;
  T* Kt = Vs + BKEY * KS;
  T* Ss = Kt + KTBUF;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int qw = blockIdx.x * 64 + w * 16;
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  const T* dO = (const T*)a.o + b * a.sob + h * a.soh;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  typename MF::frag qf[NQF], gf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s) {
    const int d = s * MF::KSTEP + (lane >> 4) * MF::KPL;
    qf[s] = frag_global<T>(Q, a.sql, qw + (lane & 15), a.Lq, d, a.D);
    gf[s] = frag_global<T>(dO, a.sol, qw + (lane & 15), a.Lq, d, a.D);
  }
  float lse2[4], di[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = qw + (lane >> 4) * 4 + r;
    lse2[r] = row < a.Lq ? a.lse[(int64_t)bh * a.Lq + row] * LOG2E : 0.f;
    di[r] = row < a.Lq ? a.di[(int64_t)bh * a.Lq + row] : 0.f;
  }
  f32x4 dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  T* Sw = Ss + w * 16 * PS;
  const int nkt = (a.Lk + BKEY - 1) / BKEY;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKEY;
    __syncthreads();
    lds_load_rows<T, BKEY, DP, KS, 256>(Ks, K, a.skl, k0, a.Lk, a.D, tid);
    lds_load_rows<T, BKEY, DP, KS, 256>(Vs, V, a.svl, k0, a.Lk, a.D, tid);
    if constexpr (!TRR) lds_load_rows_t<T, BKEY, DP, TS, 256>(Kt, K, a.skl, k0, a.Lk, a.D, tid);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NQF; ++t) {
        const int off = (j * 16 + (lane & 15)) * KS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
        s = MF::mma(qf[t], MF::load(&Ks[off]), s);
        dp = MF::mma(gf[t], MF::load(&Vs[off]), dp);
      }
      const int key = k0 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = qw + (lane >> 4) * 4 + r;
        float p = (key < a.Lk && qi < a.Lq) ? exp2f(s[r] * sl2 - lse2[r]) : 0.f;
        float g = dp[r];
        if (drop) {
          uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qi) * (uint64_t)a.Lk + key;
          g = s2h_keep(a.seed, idx, thresh) ? g * inv_keep : 0.f;
        }
        Sw[((lane >> 4) * 4 + r) * PS + j * 16 + (lane & 15)] = from_f32<T>(p * (g - di[r]));
      }
    }
    __syncthreads();
    constexpr int NPF = BKEY / MF::KSTEP;
    typename MF::frag sf[NPF];
#pragma unroll
    for (int t = 0; t < NPF; ++t) sf[t] = MF::load(&Sw[(lane & 15) * PS + t * MF::KSTEP + (lane >> 4) * MF::KPL]);
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int t = 0; t < NPF; ++t)
        dq[d] = MF::mma(sf[t], tr_or_load<T>(Ks, KS, Kt, TS, t * MF::KSTEP, d * 16, lane), dq[d]);
  }
  T* dQ = (T*)a.dq + b * a.sdqb + h * a.sdqh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = qw + (lane >> 4) * 4 + r;
    if (row < a.Lq)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int col = d * 16 + (lane & 15);
        if (col < a.D) dQ[(int64_t)row * a.sdql + col] = from_f32<T>(dq[d][r] * a.scale);
      }
  }
}

// ------------------------------------------------------ backward: dK, dV
template <typename T, int DP>
__global__ __launch_bounds__(AttnCfg<T>::NW_DKV * 64) void attn_bwd_dkv_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int NW = AttnCfg<T>::NW_DKV;
  constexpr int NT = NW * 64;
  constexpr int BQ = DkvBQ<T, DP>::v;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int KS = DP + VEC, QS = BQ + VEC;
  constexpr int NKF = DP / MF::KSTEP, NB = BQ / 16, ND = DP / 16, NPF = BQ / MF::KSTEP;
  constexpr bool TRR = sizeof(T) == 2;  // bf16: Q^T / dO^T fragments by transposing reads of Qs / Gs
  constexpr int TBUF = TRR ? 0 : DP * QS;
  __shared__ __attribute__((aligned(16))) T smem[2 * NW * 16 * KS + 2 * BQ * KS + 2 * TBUF + 2 * NW * 16 * QS];
  __shared__ float stat[2 * BQ];
  T* Kn = smem;
  T* Vn = Kn + NW * 16 * KS;
  T* Qs = Vn + NW * 16 * KS;
  T* Gs = Qs + BQ * KS;
  T* Qt = Gs + BQ * KS;
  T* Gt = Qt + TBUF;
  T* Pb = Gt + TBUF;
  T* Sb = Pb + NW * 16 * QS;
  float* lse_s = stat;
  float* di_s = stat + BQ;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int kb = blockIdx.x * NW * 16;  // first key of the workgroup
  const int kw = kb + w * 16;           // first key of this wave
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  const T* dO = (const T*)a.o + b * a.sob + h * a.soh;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  lds_load_rows<T, NW * 16, DP, KS, NT>(Kn, K, a.skl, kb, a.Lk, a.D, tid);
  lds_load_rows<T, NW * 16, DP, KS, NT>(Vn, V, a.svl, kb, a.Lk, a.D, tid);

  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }
  T* Pw = Pb + w * 16 * QS;
  T* Sw = Sb + w * 16 * QS;
  const T* Kw = Kn + w * 16 * KS;
  const T* Vw = Vn + w * 16 * KS;

  const int nqt = (a.Lq + BQ - 1) / BQ;
  for (int qt = 0; qt < nqt; ++qt) {
    const int q0 = qt * BQ;
    __syncthreads();
    lds_load_rows<T, BQ, DP, KS, NT>(Qs, Q, a.sql, q0, a.Lq, a.D, tid);
    lds_load_rows<T, BQ, DP, KS, NT>(Gs, dO, a.sol, q0, a.Lq, a.D, tid);
    if constexpr (!TRR) {
      lds_load_rows_t<T, BQ, DP, QS, NT>(Qt, Q, a.sql, q0, a.Lq, a.D, tid);
      lds_load_rows_t<T, BQ, DP, QS, NT>(Gt, dO, a.sol, q0, a.Lq, a.D, tid);
    }
    for (int i = tid; i < BQ; i += NT) {
      const int qi = q0 + i;
      lse_s[i] = qi < a.Lq ? a.lse[(int64_t)bh * a.Lq + qi] * LOG2E : 0.f;
      di_s[i] = qi < a.Lq ? a.di[(int64_t)bh * a.Lq + qi] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NKF; ++t) {
        const int ao = (lane & 15) * KS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
        const int bo = (j * 16 + (lane & 15)) * KS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
        s = MF::mma(MF::load(&Kw[ao]), MF::load(&Qs[bo]), s);
        dp = MF::mma(MF::load(&Vw[ao]), MF::load(&Gs[bo]), dp);
      }
      const int qc = j * 16 + (lane & 15);  // query column within tile
      const int qi = q0 + qc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kw + (lane >> 4) * 4 + r;
        const bool valid = key < a.Lk && qi < a.Lq;
        float p = valid ? exp2f(s[r] * sl2 - lse_s[qc]) : 0.f;
        float pd = p, g = dp[r];
        if (drop) {
          uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qi) * (uint64_t)a.Lk + key;
          bool keep = valid && s2h_keep(a.seed, idx, thresh);
          pd = keep ? p * inv_keep : 0.f;
          g = keep ? g * inv_keep : 0.f;
        }
        Pw[((lane >> 4) * 4 + r) * QS + qc] = from_f32<T>(pd);
        Sw[((lane >> 4) * 4 + r) * QS + qc] = from_f32<T>(p * (g - di_s[qc]));
      }
    }
    __syncthreads();
    typename MF::frag pf[NPF], sf[NPF];
#pragma unroll
    for (int t = 0; t < NPF; ++t) {
      const int o = (lane & 15) * QS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
      pf[t] = MF::load(&Pw[o]);
      sf[t] = MF::load(&Sw[o]);
    }
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int t = 0; t < NPF; ++t) {
        dv[d] = MF::mma(pf[t], tr_or_load<T>(Gs, KS, Gt, QS, t * MF::KSTEP, d * 16, lane), dv[d]);
        dk[d] = MF::mma(sf[t], tr_or_load<T>(Qs, KS, Qt, QS, t * MF::KSTEP, d * 16, lane), dk[d]);
      }
  }
  T* dK = (T*)a.dk + b * a.sdkb + h * a.sdkh;
  T* dV = (T*)a.dv + b * a.sdvb + h * a.sdvh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = kw + (lane >> 4) * 4 + r;
    if (key < a.Lk)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int col = d * 16 + (lane & 15);
        if (col < a.D) {
          dK[(int64_t)key * a.sdkl + col] = from_f32<T>(dk[d][r] * a.scale);
          dV[(int64_t)key * a.sdvl + col] = from_f32<T>(dv[d][r]);
        }
      }
  }
}

// ------------------------------------------- few-query / few-key specialisations
// The two-way decoder's token<->image attentions (transformer.py:231-248, 8 heads,
// head_dim 16, 8 tokens vs 1024 image rows, O*8 = 104 (batch, head) pairs) leave the
// kernels above with one useful wave per workgroup looping over the long side: 104
// workgroups, 16 serial key (or query) tiles each.  Here the 4 waves of a workgroup
// split the LONG side instead and merge their partial results in LDS at the end.
//   fwd, Lq <= 16 : waves take key tiles w, w+4, ...; partial (m, l, o) merged
//   dQ,  Lq <= 16 : waves take key tiles w, w+4, ...; partial dQ summed
//   dK/dV, Lk <= 16: waves take query tiles w, w+4, ...; partial dK, dV summed
// Loop trip counts are workgroup-uniform (an idle wave masks its tile) so the barriers
// are safe.  K / Q rows feed the MFMA B operand straight from global (16-B loads); only
// the operands that need a transposed (key-major or query-major) fragment go through
// wave-private LDS.
// sum of the NW waves' partials of one element (stride = floats per wave's partial block)
template <int NW>
__device__ __forceinline__ float mrg_sum(const float* p, int stride) {
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NW; ++u) s += p[u * stride];
  return s;
}

template <typename T, int DP, int NW = 4>
__global__ __launch_bounds__(NW * 64) void attn_fwd_fewq_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int BKEY = 64;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int VS = BKEY + VEC, PS = BKEY + VEC;
  constexpr int NQF = DP / MF::KSTEP, NB = BKEY / 16, ND = DP / 16, NPF = BKEY / MF::KSTEP;
  constexpr int WL = DP * VS + 16 * PS;  // wave-private LDS elements
  __shared__ __attribute__((aligned(16))) T smem[NW * WL];
  __shared__ float mrg[NW][16][DP + 2];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  T* Vt = smem + w * WL;
  T* Pw = Vt + DP * VS;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  typename MF::frag qf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s)
    qf[s] = frag_global<T>(Q, a.sql, lane & 15, a.Lq, s * MF::KSTEP + (lane >> 4) * MF::KPL, a.D);
  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -INFINITY; l[r] = 0.f; }

  const int nkt = (a.Lk + BKEY - 1) / BKEY;
  for (int it = 0; it < (nkt + NW - 1) / NW; ++it) {
    const int kt = it * NW + w;
    const int k0 = kt * BKEY;
    if (kt < nkt) {
      lds_load_rows_t<T, BKEY, DP, VS, 64>(Vt, V, a.svl, k0, a.Lk, a.D, lane);
      f32x4 s[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NQF; ++t)
          s[j] = MF::mma(qf[t], frag_global<T>(K, a.skl, k0 + j * 16 + (lane & 15), a.Lk,
                                               t * MF::KSTEP + (lane >> 4) * MF::KPL, a.D), s[j]);
      }
      float mx[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bool kvalid = k0 + j * 16 + (lane & 15) < a.Lk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = kvalid ? s[j][r] * sl2 : -INFINITY;
          s[j][r] = x;
          mx[r] = fmaxf(mx[r], x);
        }
      }
      float alpha[4], rs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mx[r] = row16_max(mx[r]);
        const float mn = fmaxf(m[r], mx[r]);
        alpha[r] = exp2f(m[r] - mn);
        m[r] = mn;
        rs[r] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int key = k0 + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = exp2f(s[j][r] - m[r]);
          rs[r] += p;
          if (drop) {
            const int qi = (lane >> 4) * 4 + r;
            const uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qi) * (uint64_t)a.Lk + key;
            p = s2h_keep(a.seed, idx, thresh) ? p * inv_keep : 0.f;
          }
          Pw[((lane >> 4) * 4 + r) * PS + j * 16 + (lane & 15)] = from_f32<T>(p);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) l[r] = l[r] * alpha[r] + row16_sum(rs[r]);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d][r] *= alpha[r];
    }
    __syncthreads();  // this wave's Vt / Pw writes visible to its own fragment reads
    if (kt < nkt) {
      typename MF::frag pf[NPF];
#pragma unroll
      for (int t = 0; t < NPF; ++t) pf[t] = MF::load(&Pw[(lane & 15) * PS + t * MF::KSTEP + (lane >> 4) * MF::KPL]);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int t = 0; t < NPF; ++t)
          o[d] = MF::mma(pf[t], MF::load(&Vt[(d * 16 + (lane & 15)) * VS + t * MF::KSTEP + (lane >> 4) * MF::KPL]),
                         o[d]);
    }
    __syncthreads();  // reads done before the next tile overwrites Vt / Pw
  }
  // merge the 4 waves' (m, l, o)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) * 4 + r;
#pragma unroll
    for (int d = 0; d < ND; ++d) mrg[w][row][d * 16 + (lane & 15)] = o[d][r];
    if ((lane & 15) == 0) { mrg[w][row][DP] = m[r]; mrg[w][row][DP + 1] = l[r]; }
  }
  __syncthreads();
  T* O = (T*)a.o + b * a.sob + h * a.soh;
  for (int e = tid; e < 16 * DP; e += NW * 64) {
    const int row = e / DP, col = e % DP;
    if (row >= a.Lq) continue;
    float M = -INFINITY;
#pragma unroll
    for (int u = 0; u < NW; ++u) M = fmaxf(M, mrg[u][row][DP]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const float f = exp2f(mrg[u][row][DP] - M);  // waves without keys: m = -inf -> 0
      L += mrg[u][row][DP + 1] * f;
      acc += mrg[u][row][col] * f;
    }
    if (col < a.D) O[(int64_t)row * a.sol + col] = from_f32<T>(acc / L);
    if (col == 0) a.lse[(int64_t)bh * a.Lq + row] = (M + log2f(L)) * LN2;
  }
}

template <typename T, int DP, int NW = 4>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dq_fewq_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int BKEY = 64;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int TS = BKEY + VEC, PS = BKEY + VEC;
  constexpr int NQF = DP / MF::KSTEP, NB = BKEY / 16, ND = DP / 16, NPF = BKEY / MF::KSTEP;
  constexpr int WL = DP * TS + 16 * PS;
  __shared__ __attribute__((aligned(16))) T smem[NW * WL];
  __shared__ float mrg[NW][16][DP + 1];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  const T* dO = (const T*)a.o + b * a.sob + h * a.soh;
  T* Kt = smem + w * WL;
  T* Sw = Kt + DP * TS;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  typename MF::frag qf[NQF], gf[NQF];
#pragma unroll
  for (int s = 0; s < NQF; ++s) {
    const int d = s * MF::KSTEP + (lane >> 4) * MF::KPL;
    qf[s] = frag_global<T>(Q, a.sql, lane & 15, a.Lq, d, a.D);
    gf[s] = frag_global<T>(dO, a.sol, lane & 15, a.Lq, d, a.D);
  }
  float lse2[4], di[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) * 4 + r;
    lse2[r] = row < a.Lq ? a.lse[(int64_t)bh * a.Lq + row] * LOG2E : 0.f;
    di[r] = row < a.Lq ? a.di[(int64_t)bh * a.Lq + row] : 0.f;
  }
  f32x4 dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (a.Lk + BKEY - 1) / BKEY;
  for (int it = 0; it < (nkt + NW - 1) / NW; ++it) {
    const int kt = it * NW + w;
    const int k0 = kt * BKEY;
    if (kt < nkt) {
      lds_load_rows_t<T, BKEY, DP, TS, 64>(Kt, K, a.skl, k0, a.Lk, a.D, lane);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
        const int krow = k0 + j * 16 + (lane & 15);
#pragma unroll
        for (int t = 0; t < NQF; ++t) {
          const int d = t * MF::KSTEP + (lane >> 4) * MF::KPL;
          s = MF::mma(qf[t], frag_global<T>(K, a.skl, krow, a.Lk, d, a.D), s);
          dp = MF::mma(gf[t], frag_global<T>(V, a.svl, krow, a.Lk, d, a.D), dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = (lane >> 4) * 4 + r;
          const float p = (krow < a.Lk && qi < a.Lq) ? exp2f(s[r] * sl2 - lse2[r]) : 0.f;
          float g = dp[r];
          if (drop) {
            const uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qi) * (uint64_t)a.Lk + krow;
            g = s2h_keep(a.seed, idx, thresh) ? g * inv_keep : 0.f;
          }
          Sw[((lane >> 4) * 4 + r) * PS + j * 16 + (lane & 15)] = from_f32<T>(p * (g - di[r]));
        }
      }
    }
    __syncthreads();
    if (kt < nkt) {
      typename MF::frag sf[NPF];
#pragma unroll
      for (int t = 0; t < NPF; ++t) sf[t] = MF::load(&Sw[(lane & 15) * PS + t * MF::KSTEP + (lane >> 4) * MF::KPL]);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int t = 0; t < NPF; ++t)
          dq[d] = MF::mma(sf[t], MF::load(&Kt[(d * 16 + (lane & 15)) * TS + t * MF::KSTEP + (lane >> 4) * MF::KPL]),
                          dq[d]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int d = 0; d < ND; ++d) mrg[w][(lane >> 4) * 4 + r][d * 16 + (lane & 15)] = dq[d][r];
  __syncthreads();
  T* dQ = (T*)a.dq + b * a.sdqb + h * a.sdqh;
  for (int e = tid; e < 16 * DP; e += NW * 64) {
    const int row = e / DP, col = e % DP;
    if (row < a.Lq && col < a.D)
      dQ[(int64_t)row * a.sdql + col] =
          from_f32<T>(mrg_sum<NW>(&mrg[0][row][col], 16 * (DP + 1)) * a.scale);
  }
}

template <typename T, int DP, int NW = 4>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dkv_fewk_kernel(AttnArgs a) {
  if (a.p_drop > 0.f) a.seed = s2h_seed(a.seed, a.seed_off);
  using MF = Mfma<T>;
  constexpr int BQ = sizeof(T) == 2 ? 64 : 32;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int KS = DP + VEC, QS = BQ + VEC;
  constexpr int NKF = DP / MF::KSTEP, NB = BQ / 16, ND = DP / 16, NPF = BQ / MF::KSTEP;
  constexpr int WL = 2 * DP * QS + 2 * 16 * QS;
  __shared__ __attribute__((aligned(16))) T smem[2 * 16 * KS + NW * WL];
  __shared__ float stat[NW][2 * BQ];
  __shared__ float mrg[NW][16][2 * DP];
  T* Kn = smem;
  T* Vn = Kn + 16 * KS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  T* Qt = Vn + 16 * KS + w * WL;
  T* Gt = Qt + DP * QS;
  T* Pw = Gt + DP * QS;
  T* Sw = Pw + 16 * QS;
  float* lse_s = stat[w];
  float* di_s = stat[w] + BQ;

  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const T* Q = (const T*)a.q + b * a.sqb + h * a.sqh;
  const T* K = (const T*)a.k + b * a.skb + h * a.skh;
  const T* V = (const T*)a.v + b * a.svb + h * a.svh;
  const T* dO = (const T*)a.o + b * a.sob + h * a.soh;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.p_drop > 0.f;
  const uint32_t thresh = (uint32_t)(a.p_drop * 4294967296.0);
  const float inv_keep = drop ? 1.f / (1.f - a.p_drop) : 1.f;

  lds_load_rows<T, 16, DP, KS, NW * 64>(Kn, K, a.skl, 0, a.Lk, a.D, tid);
  lds_load_rows<T, 16, DP, KS, NW * 64>(Vn, V, a.svl, 0, a.Lk, a.D, tid);
  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }

  const int nqt = (a.Lq + BQ - 1) / BQ;
  for (int it = 0; it < (nqt + NW - 1) / NW; ++it) {
    const int qt = it * NW + w;
    const int q0 = qt * BQ;
    __syncthreads();  // Kn/Vn loaded (first pass); previous tile's reads done
    if (qt < nqt) {
      lds_load_rows_t<T, BQ, DP, QS, 64>(Qt, Q, a.sql, q0, a.Lq, a.D, lane);
      lds_load_rows_t<T, BQ, DP, QS, 64>(Gt, dO, a.sol, q0, a.Lq, a.D, lane);
      for (int i = lane; i < BQ; i += 64) {
        const int qi = q0 + i;
        lse_s[i] = qi < a.Lq ? a.lse[(int64_t)bh * a.Lq + qi] * LOG2E : 0.f;
        di_s[i] = qi < a.Lq ? a.di[(int64_t)bh * a.Lq + qi] : 0.f;
      }
    }
    __syncthreads();
    if (qt < nqt) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
        const int qrow = q0 + j * 16 + (lane & 15);
#pragma unroll
        for (int t = 0; t < NKF; ++t) {
          const int ao = (lane & 15) * KS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
          const int d = t * MF::KSTEP + (lane >> 4) * MF::KPL;
          s = MF::mma(MF::load(&Kn[ao]), frag_global<T>(Q, a.sql, qrow, a.Lq, d, a.D), s);
          dp = MF::mma(MF::load(&Vn[ao]), frag_global<T>(dO, a.sol, qrow, a.Lq, d, a.D), dp);
        }
        const int qc = j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = (lane >> 4) * 4 + r;
          const bool valid = key < a.Lk && qrow < a.Lq;
          const float p = valid ? exp2f(s[r] * sl2 - lse_s[qc]) : 0.f;
          float pd = p, g = dp[r];
          if (drop) {
            const uint64_t idx = a.idx0 + ((uint64_t)bh * a.Lq + qrow) * (uint64_t)a.Lk + key;
            const bool keep = valid && s2h_keep(a.seed, idx, thresh);
            pd = keep ? p * inv_keep : 0.f;
            g = keep ? g * inv_keep : 0.f;
          }
          Pw[key * QS + qc] = from_f32<T>(pd);
          Sw[key * QS + qc] = from_f32<T>(p * (g - di_s[qc]));
        }
      }
    }
    __syncthreads();
    if (qt < nqt) {
      typename MF::frag pf[NPF], sf[NPF];
#pragma unroll
      for (int t = 0; t < NPF; ++t) {
        const int o = (lane & 15) * QS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
        pf[t] = MF::load(&Pw[o]);
        sf[t] = MF::load(&Sw[o]);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int t = 0; t < NPF; ++t) {
          const int o = (d * 16 + (lane & 15)) * QS + t * MF::KSTEP + (lane >> 4) * MF::KPL;
          dv[d] = MF::mma(pf[t], MF::load(&Gt[o]), dv[d]);
          dk[d] = MF::mma(sf[t], MF::load(&Qt[o]), dk[d]);
        }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      mrg[w][(lane >> 4) * 4 + r][d * 16 + (lane & 15)] = dk[d][r];
      mrg[w][(lane >> 4) * 4 + r][DP + d * 16 + (lane & 15)] = dv[d][r];
    }
  __syncthreads();
  T* dK = (T*)a.dk + b * a.sdkb + h * a.sdkh;
  T* dV = (T*)a.dv + b * a.sdvb + h * a.sdvh;
  for (int e = tid; e < 16 * DP; e += NW * 64) {
    const int key = e / DP, col = e % DP;
    if (key < a.Lk && col < a.D) {
      const float sk = mrg_sum<NW>(&mrg[0][key][col], 16 * 2 * DP);
      const float sv = mrg_sum<NW>(&mrg[0][key][DP + col], 16 * 2 * DP);
      dK[(int64_t)key * a.sdkl + col] = from_f32<T>(sk * a.scale);
      dV[(int64_t)key * a.sdvl + col] = from_f32<T>(sv);
    }
  }
}

// ------------------------------------------------- small windows (Lq, Lk <= 64)
// Hiera's windowed and q-pooled attentions (hieradet.py:56-81: 8x8 / 4x4 windows, 2x2-pooled
// queries, the 7x7 global stage) are 10^3-10^4 independent (window, head) instances of at most
// 64 x 64.  The tile kernels above give every instance a 64-query x 64-key workgroup (a 4x4
// window uses 1/16 of it) and the backward three launches (Di, dQ, dK / dV).  Here a workgroup
// owns whole instances: Lq <= 16 -> one wave (64 threads) per instance, Lq <= 64 -> four waves
// of 16 query rows.  The keys are one LDS tile of KR (32 / 64) rows, so the softmax is exact in
// one pass; the backward computes P, dP, Di = rowsum(P o dP) (= rowsum(dO o O) of the exact
// forward), dS and dQ in the query waves, then dK / dV per 16-key block from P and dS kept in
// LDS -- one launch, no atomics, no workspace.  bf16, head dim <= 64 (zero-padded image of 64),
// no dropout (Hiera has none; dropout sites keep the tile kernels).
// MFMA fragment maps (16x16x32 bf16): A[m][k] / B[n][k] -> lane (m | n = lane & 15, k = 8 (lane >> 4)
// .. +7); C -> lane (row 4 (lane >> 4) + r, col lane & 15).  A "k-major" image [k][m] gives the
// fragment by transposing reads (tr_bfrag), a row-major one [m][k] by ds_read_b128.
constexpr int WIN_DP = 64, WIN_KS = WIN_DP + 8;

template <int NW, int KR>
__global__ __launch_bounds__(NW * 64) void attn_win_fwd_kernel(AttnArgs a) {
  using MF = Mfma<bf16>;
  constexpr int KS = WIN_KS, PS = KR + 8, QR = 16 * NW, NT = NW * 64, NB = KR / 16;
  // K feeds S = Q K^T only (B operand in its natural layout): fragments straight from global
  __shared__ __attribute__((aligned(16))) bf16 smem[KR * KS + QR * PS + QR * KS];
  bf16* Vs = smem;
  bf16* Ps = Vs + KR * KS;
  bf16* Os = Ps + QR * PS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const bf16* Q = (const bf16*)a.q + b * a.sqb + h * a.sqh;
  const bf16* K = (const bf16*)a.k + b * a.skb + h * a.skh;
  const bf16* V = (const bf16*)a.v + b * a.svb + h * a.svh;
  const int q0 = blockIdx.y * QR + 16 * w;  // query tiles of QR rows (Lq > 64: the decoder's image -> token)
  MF::frag qf[2], kf[NB][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    qf[t] = frag_global<bf16>(Q, a.sql, q0 + (lane & 15), a.Lq, t * 32 + (lane >> 4) * 8, a.D);
#pragma unroll
    for (int j = 0; j < NB; ++j) kf[j][t] = frag_global<bf16>(K, a.skl, j * 16 + (lane & 15), a.Lk, t * 32 + (lane >> 4) * 8, a.D);
  }
  lds_load_rows<bf16, KR, WIN_DP, KS, NT>(Vs, V, a.svl, 0, a.Lk, a.D, tid);

  const float sl2 = a.scale * LOG2E;
  f32x4 s[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) s[j] = MF::mma(qf[t], kf[j][t], s[j]);
  }
  float mx[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const bool kvalid = j * 16 + (lane & 15) < a.Lk;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[j][r] = kvalid ? s[j][r] * sl2 : -INFINITY;
      mx[r] = fmaxf(mx[r], s[j][r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mx[r] = row16_max(mx[r]);
    l[r] = 0.f;
  }
  bf16* Pw = Ps + 16 * w * PS;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = exp2f(s[j][r] - mx[r]);
      l[r] += p;
      Pw[(4 * (lane >> 4) + r) * PS + j * 16 + (lane & 15)] = (bf16)p;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) l[r] = row16_sum(l[r]);
  __syncthreads();  // the V tile (all waves' loads); P rows are this wave's own
  f32x4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KR / 32; ++t) {
    const MF::frag pf = MF::load(&Pw[(lane & 15) * PS + t * 32 + (lane >> 4) * 8]);
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = MF::mma(pf, tr_bfrag(Vs, KS, t * 32, d * 16, lane), o[d]);
  }
  bf16* Ow = Os + 16 * w * KS;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / l[r];
#pragma unroll
    for (int d = 0; d < 4; ++d) Ow[(4 * (lane >> 4) + r) * KS + d * 16 + (lane & 15)] = (bf16)(o[d][r] * inv);
    const int row = q0 + 4 * (lane >> 4) + r;
    if ((lane & 15) == 0 && row < a.Lq) a.lse[(int64_t)bh * a.Lq + row] = (mx[r] + log2f(l[r])) * LN2;
  }
  bf16* O = (bf16*)a.o + b * a.sob + h * a.soh;
#pragma unroll
  for (int c = lane; c < 16 * 8; c += 64) {  // 16 rows x 8 16-B chunks of this wave's output
    const int row = c >> 3, col = (c & 7) * 8;
    if (q0 + row < a.Lq && col < a.D) *(uint4*)(O + (int64_t)(q0 + row) * a.sol + col) = *(const uint4*)(Ow + row * KS + col);
  }
}

// 16x16x16 operand (k = 4 (lane >> 4) .. +3) from a k-major [k][m] image: one transposing read
__device__ __forceinline__ attn_v4i16 tr_bfrag16(const bf16* img, int ld, int k0, int n0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) attn_v4i16 lds_v4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + (k0 + 4 * g + q) * ld + n0 + 4 * p));
}

// V only feeds dP = dO V^T (B operand in its natural [key][d] layout): its fragments come straight
// from global, so LDS holds K, Q, dO, P and dS.  One-wave instances (Lq <= 16) reduce dK / dV over
// their 16 query rows with the 16-deep MFMA (no zero rows padding the reduction to 32): 11.8 /
// 18.4 KB of LDS per instance at KR = 32 / 64, i.e. 13 / 8 instances resident per CU.
template <int NW, int KR>
__global__ __launch_bounds__(NW * 64) void attn_win_bwd_kernel(AttnArgs a) {
  using MF = Mfma<bf16>;
  constexpr int KS = WIN_KS, PS = KR + 8, QA = 16 * NW, NT = NW * 64, NB = KR / 16;
  constexpr bool X16 = NW == 1;
  __shared__ __attribute__((aligned(16))) bf16 smem[KR * KS + 2 * QA * KS + 2 * QA * PS];
  bf16* Ks = smem;
  bf16* Qs = Ks + KR * KS;
  bf16* Gs = Qs + QA * KS;  // dO
  bf16* Ps = Gs + QA * KS;
  bf16* Ss = Ps + QA * PS;  // dS
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const bf16* V = (const bf16*)a.v + b * a.svb + h * a.svh;
  MF::frag vf[NB][2];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int t = 0; t < 2; ++t) vf[j][t] = frag_global<bf16>(V, a.svl, j * 16 + (lane & 15), a.Lk, t * 32 + (lane >> 4) * 8, a.D);
  lds_load_rows<bf16, KR, WIN_DP, KS, NT>(Ks, (const bf16*)a.k + b * a.skb + h * a.skh, a.skl, 0, a.Lk, a.D, tid);
  lds_load_rows<bf16, QA, WIN_DP, KS, NT>(Qs, (const bf16*)a.q + b * a.sqb + h * a.sqh, a.sql, 0, a.Lq, a.D, tid);
  lds_load_rows<bf16, QA, WIN_DP, KS, NT>(Gs, (const bf16*)a.o + b * a.sob + h * a.soh, a.sol, 0, a.Lq, a.D, tid);
  const int q0 = 16 * w;
  const float sl2 = a.scale * LOG2E;
  float lse2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = q0 + 4 * (lane >> 4) + r;
    lse2[r] = row < a.Lq ? a.lse[(int64_t)bh * a.Lq + row] * LOG2E : 0.f;
  }
  __syncthreads();

  // query phase: P, dP, Di, dS of rows q0 .. q0 + 15; dQ = dS K
  f32x4 s[NB], dp[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ao = (q0 + (lane & 15)) * KS + t * 32 + (lane >> 4) * 8;
      s[j] = MF::mma(MF::load(&Qs[ao]), MF::load(&Ks[(j * 16 + (lane & 15)) * KS + t * 32 + (lane >> 4) * 8]), s[j]);
      dp[j] = MF::mma(MF::load(&Gs[ao]), vf[j][t], dp[j]);
    }
  }
  float di[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const bool kvalid = j * 16 + (lane & 15) < a.Lk;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool qvalid = q0 + 4 * (lane >> 4) + r < a.Lq;
      s[j][r] = (kvalid && qvalid) ? exp2f(s[j][r] * sl2 - lse2[r]) : 0.f;  // P
      di[r] += s[j][r] * dp[j][r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) di[r] = row16_sum(di[r]);
  bf16* Pw = Ps + q0 * PS;
  bf16* Sw = Ss + q0 * PS;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int at = (4 * (lane >> 4) + r) * PS + j * 16 + (lane & 15);
      Pw[at] = (bf16)s[j][r];
      Sw[at] = (bf16)(s[j][r] * (dp[j][r] - di[r]));
    }
  f32x4 dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KR / 32; ++t) {
    const MF::frag sf = MF::load(&Sw[(lane & 15) * PS + t * 32 + (lane >> 4) * 8]);
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[d] = MF::mma(sf, tr_bfrag(Ks, KS, t * 32, d * 16, lane), dq[d]);
  }
  bf16* dQ = (bf16*)a.dq + b * a.sdqb + h * a.sdqh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = q0 + 4 * (lane >> 4) + r;
    if (row < a.Lq)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int col = d * 16 + (lane & 15);
        if (col < a.D) dQ[(int64_t)row * a.sdql + col] = (bf16)(dq[d][r] * a.scale);
      }
  }
  __syncthreads();

  // key phase: dV = P^T dO, dK = dS^T Q per 16-key block (reductions over all QA query rows)
  bf16* dK = (bf16*)a.dk + b * a.sdkb + h * a.sdkh;
  bf16* dV = (bf16*)a.dv + b * a.sdvb + h * a.sdvh;
  for (int kb = w; kb < NB; kb += NW) {
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (X16) {
      const attn_v4i16 pt = tr_bfrag16(Ps, PS, 0, kb * 16, lane);
      const attn_v4i16 st = tr_bfrag16(Ss, PS, 0, kb * 16, lane);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        dv[d] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pt, tr_bfrag16(Gs, KS, 0, d * 16, lane), dv[d], 0, 0, 0);
        dk[d] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(st, tr_bfrag16(Qs, KS, 0, d * 16, lane), dk[d], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < QA / 32; ++t) {
        const MF::frag pt = tr_bfrag(Ps, PS, t * 32, kb * 16, lane);
        const MF::frag st = tr_bfrag(Ss, PS, t * 32, kb * 16, lane);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          dv[d] = MF::mma(pt, tr_bfrag(Gs, KS, t * 32, d * 16, lane), dv[d]);
          dk[d] = MF::mma(st, tr_bfrag(Qs, KS, t * 32, d * 16, lane), dk[d]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kb * 16 + 4 * (lane >> 4) + r;
      if (key < a.Lk)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int col = d * 16 + (lane & 15);
          if (col < a.D) {
            dK[(int64_t)key * a.sdkl + col] = (bf16)(dk[d][r] * a.scale);
            dV[(int64_t)key * a.sdvl + col] = (bf16)dv[d][r];
          }
        }
    }
  }
}

// dK / dV of a few-query attention (Lq <= 16 against a long key side: the decoder's token -> image
// attention, 8 tokens x 1024 image keys, head dim 16): per 64-key block, 4 waves of 16 keys compute
// S^T = K Q^T and dP^T = V dO^T (keys on the MFMA rows, K / V fragments straight from global),
// P^T and dS^T = P^T o (dP^T - Di) with the forward's LSE and the pre-pass Di of each query column,
// then dV = P^T dO and dK = dS^T Q with the 16-deep MFMA over the query axis (P^T / dS^T through a
// wave-private LDS slab, Q / dO k-major images read transposed).  The tile kernel ran each 64-key
// block against a 64-query tile with 8 valid rows.
template <int DP>
__global__ __launch_bounds__(256) void attn_fewq_dkv_kernel(AttnArgs a) {
  using MF = Mfma<bf16>;
  constexpr int KS = DP + 8, QS = 16 + 8, NKT = DP / 32, ND = DP / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 16 * KS + 2 * 4 * 16 * QS];
  bf16* Qs = smem;
  bf16* Gs = Qs + 16 * KS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16* PT = Gs + 16 * KS + w * 2 * 16 * QS;  // this wave's P^T [key][q]
  bf16* ST = PT + 16 * QS;                     // and dS^T
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int k0 = blockIdx.x * 64 + 16 * w;
  lds_load_rows<bf16, 16, DP, KS, 256>(Qs, (const bf16*)a.q + b * a.sqb + h * a.sqh, a.sql, 0, a.Lq, a.D, tid);
  lds_load_rows<bf16, 16, DP, KS, 256>(Gs, (const bf16*)a.o + b * a.sob + h * a.soh, a.sol, 0, a.Lq, a.D, tid);
  const bf16* K = (const bf16*)a.k + b * a.skb + h * a.skh;
  const bf16* V = (const bf16*)a.v + b * a.svb + h * a.svh;
  MF::frag kf[NKT], vf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    kf[t] = frag_global<bf16>(K, a.skl, k0 + (lane & 15), a.Lk, t * 32 + (lane >> 4) * 8, a.D);
    vf[t] = frag_global<bf16>(V, a.svl, k0 + (lane & 15), a.Lk, t * 32 + (lane >> 4) * 8, a.D);
  }
  const int q = lane & 15;
  const bool qok = q < a.Lq;
  const float lse2 = qok ? a.lse[(int64_t)bh * a.Lq + q] * LOG2E : 0.f;
  const float di = qok ? a.di[(int64_t)bh * a.Lq + q] : 0.f;
  const float sl2 = a.scale * LOG2E;
  __syncthreads();
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int bo = q * KS + t * 32 + (lane >> 4) * 8;
    s = MF::mma(kf[t], MF::load(&Qs[bo]), s);
    dp = MF::mma(vf[t], MF::load(&Gs[bo]), dp);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kl = 4 * (lane >> 4) + r;
    const float p = (qok && k0 + kl < a.Lk) ? exp2f(s[r] * sl2 - lse2) : 0.f;
    PT[kl * QS + q] = (bf16)p;
    ST[kl * QS + q] = (bf16)(p * (dp[r] - di));
  }
  // dV = P^T dO, dK = dS^T Q over the 16 query rows (rows >= Lq are zero in Qs / Gs and in P^T)
  typedef short v4s __attribute__((ext_vector_type(4)));
  const v4s pa = *(const v4s*)&PT[(lane & 15) * QS + 4 * (lane >> 4)];
  const v4s sa = *(const v4s*)&ST[(lane & 15) * QS + 4 * (lane >> 4)];
  bf16* dK = (bf16*)a.dk + b * a.sdkb + h * a.sdkh;
  bf16* dV = (bf16*)a.dv + b * a.sdvb + h * a.sdvh;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 dv = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, tr_bfrag16(Gs, KS, 0, d * 16, lane), z, 0, 0, 0);
    const f32x4 dk = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(sa, tr_bfrag16(Qs, KS, 0, d * 16, lane), z, 0, 0, 0);
    const int col = d * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + 4 * (lane >> 4) + r;
      if (key < a.Lk && col < a.D) {
        dK[(int64_t)key * a.sdkl + col] = (bf16)(dk[r] * a.scale);
        dV[(int64_t)key * a.sdvl + col] = (bf16)dv[r];
      }
    }
  }
}

// dQ of a few-key attention (Lk <= 16 against a long query side: the decoder's image -> token
// attention, 1024 image queries x 8 tokens): per 64-query block, 4 waves of 16 queries compute S, dP
// against the one 16-key tile (K / V fragments shared from LDS / registers), dS = P o (dP - Di), and
// dQ = dS K with the 16-deep MFMA over the key axis (dS through a wave-private LDS slab, K read
// transposed).  The tile kernel paired each 64-query tile with a 64-key tile of 8 valid keys.
template <int DP>
__global__ __launch_bounds__(256) void attn_fewk_dq_kernel(AttnArgs a) {
  using MF = Mfma<bf16>;
  constexpr int KS = DP + 8, SS = 16 + 8, NKT = DP / 32, ND = DP / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[16 * KS + 8 * 16 * SS];
  bf16* Ks = smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16* Sw = Ks + 16 * KS + w * 2 * 16 * SS;  // this wave's dS [q][key]: bf16 high part, then the residual
  bf16* Sl = Sw + 16 * SS;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int q0 = blockIdx.x * 64 + 16 * w;
  const bf16* K = (const bf16*)a.k + b * a.skb + h * a.skh;
  const bf16* V = (const bf16*)a.v + b * a.svb + h * a.svh;
  const bf16* Q = (const bf16*)a.q + b * a.sqb + h * a.sqh;
  const bf16* dO = (const bf16*)a.o + b * a.sob + h * a.soh;
  lds_load_rows<bf16, 16, DP, KS, 256>(Ks, K, a.skl, 0, a.Lk, a.D, tid);
  MF::frag qf[NKT], gf[NKT], kf[NKT], vf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int d = t * 32 + (lane >> 4) * 8;
    qf[t] = frag_global<bf16>(Q, a.sql, q0 + (lane & 15), a.Lq, d, a.D);
    gf[t] = frag_global<bf16>(dO, a.sol, q0 + (lane & 15), a.Lq, d, a.D);
    kf[t] = frag_global<bf16>(K, a.skl, lane & 15, a.Lk, d, a.D);
    vf[t] = frag_global<bf16>(V, a.svl, lane & 15, a.Lk, d, a.D);
  }
  float lse2[4], di[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = q0 + 4 * (lane >> 4) + r;
    lse2[r] = row < a.Lq ? a.lse[(int64_t)bh * a.Lq + row] * LOG2E : 0.f;
    di[r] = row < a.Lq ? a.di[(int64_t)bh * a.Lq + row] : 0.f;
  }
  const float sl2 = a.scale * LOG2E;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    s = MF::mma(qf[t], kf[t], s);
    dp = MF::mma(gf[t], vf[t], dp);
  }
  const bool kok = (lane & 15) < a.Lk;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool qok = q0 + 4 * (lane >> 4) + r < a.Lq;
    const float p = (kok && qok) ? exp2f(s[r] * sl2 - lse2[r]) : 0.f;
    const float ds = p * (dp[r] - di[r]);
    const bf16 hi = (bf16)ds;
    Sw[(4 * (lane >> 4) + r) * SS + (lane & 15)] = hi;
    Sl[(4 * (lane >> 4) + r) * SS + (lane & 15)] = (bf16)(ds - (float)hi);
  }
  __syncthreads();  // the K tile (all waves' loads); dS rows are this wave's own
  // dQ = dS K with dS as a bf16 pair (high part + rounding residual, two MFMAs at Lk <= 16): dQ
  // carries dS to fp32-accumulation precision before its one bf16 rounding
  typedef short v4s __attribute__((ext_vector_type(4)));
  const v4s sa = *(const v4s*)&Sw[(lane & 15) * SS + 4 * (lane >> 4)];
  const v4s sl = *(const v4s*)&Sl[(lane & 15) * SS + 4 * (lane >> 4)];
  bf16* dQ = (bf16*)a.dq + b * a.sdqb + h * a.sdqh;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const auto kb = tr_bfrag16(Ks, KS, 0, d * 16, lane);
    f32x4 dq = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(sl, kb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    dq = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(sa, kb, dq, 0, 0, 0);
    const int col = d * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = q0 + 4 * (lane >> 4) + r;
      if (row < a.Lq && col < a.D) dQ[(int64_t)row * a.sdql + col] = (bf16)(dq[r] * a.scale);
    }
  }
}

// A/B knob (s2h_attn_win): 0 keeps the small windows on the tile kernels
static int g_attn_win = 1;
extern "C" int s2h_attn_win(int on) {
  const int prev = g_attn_win;
  g_attn_win = on;
  return prev;
}
// the forward also takes Lq > 64 (query tiles on grid.y: the decoder's image -> token attention,
// 1024 queries x 8 keys); the one-launch backward needs every query of an instance in one workgroup
static bool attn_win_ok(const AttnArgs& a, bool fwd) {
  return g_attn_win && a.p_drop <= 0.f && a.D <= WIN_DP && (fwd ? a.Lq <= 65535 * 64 : a.Lq <= 64) && a.Lk <= 64;
}
template <bool FWD>
static int attn_win_launch(const AttnArgs& a, hipStream_t st) {
  const int slot = s2h_prof_begin(st, FWD ? 1 : 2, (int64_t)a.B * a.H, a.Lq, a.Lk, a.D, 2);
  const dim3 grid(a.B * a.H, a.Lq <= 16 ? 1 : (a.Lq + 63) / 64);
  const bool k32 = a.Lk <= 32;
  if (a.Lq <= 16) {
    if (FWD) {
      if (k32) hipLaunchKernelGGL((attn_win_fwd_kernel<1, 32>), grid, dim3(64), 0, st, a);
      else hipLaunchKernelGGL((attn_win_fwd_kernel<1, 64>), grid, dim3(64), 0, st, a);
    } else {
      if (k32) hipLaunchKernelGGL((attn_win_bwd_kernel<1, 32>), grid, dim3(64), 0, st, a);
      else hipLaunchKernelGGL((attn_win_bwd_kernel<1, 64>), grid, dim3(64), 0, st, a);
    }
  } else {
    if (FWD) {
      if (k32) hipLaunchKernelGGL((attn_win_fwd_kernel<4, 32>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_win_fwd_kernel<4, 64>), grid, dim3(256), 0, st, a);
    } else {
      if (k32) hipLaunchKernelGGL((attn_win_bwd_kernel<4, 32>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_win_bwd_kernel<4, 64>), grid, dim3(256), 0, st, a);
    }
  }
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ launch
// few-query / few-key paths pay off when the long side spans several 64-row tiles
static bool attn_fewq(const AttnArgs& a) { return a.Lq <= 16 && a.Lk > 128 && a.D <= 64; }
static bool attn_fewk(const AttnArgs& a) { return a.Lk <= 16 && a.Lq > 128 && a.D <= 64; }

template <typename T, int DP>
static int attn_fwd_launch(const AttnArgs& a, hipStream_t st) {
  dim3 grid((a.Lq + 63) / 64, a.B * a.H);
  const int slot = s2h_prof_begin(st, 1, (int64_t)a.B * a.H, a.Lq, a.Lk, a.D, sizeof(T));
  if constexpr (DP <= 64) {
    if (attn_fewq(a)) {
      // bf16 head dim <= 16 (the decoder's 8 heads x 16): 16 waves, one 64-key tile each at Lk 1024
      if constexpr (sizeof(T) == 2 && DP == 32) hipLaunchKernelGGL((attn_fwd_fewq_kernel<T, DP, 16>), dim3(a.B * a.H), dim3(1024), 0, st, a);
      else hipLaunchKernelGGL((attn_fwd_fewq_kernel<T, DP>), dim3(a.B * a.H), dim3(256), 0, st, a);
      s2h_prof_end(slot, st);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((attn_fwd_kernel<T, DP>), grid, dim3(256), 0, st, a);
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}
template <typename T, int DP>
static int attn_bwd_launch(const AttnArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.H * a.Lq;
  const int slot = s2h_prof_begin(st, 2, (int64_t)a.B * a.H, a.Lq, a.Lk, a.D, sizeof(T));
  {
    constexpr int V = 16 / sizeof(T);
    auto al = [](const void* p, int64_t s1, int64_t s2, int64_t s3) {
      return (uintptr_t)p % 16 == 0 && s1 % V == 0 && s2 % V == 0 && s3 % V == 0;
    };
    const int vec = a.D % V == 0 && al(a.o, a.sob, a.soh, a.sol) && al(a.fo, a.sfb, a.sfh, a.sfl);
    const int per = vec ? (a.D + V - 1) / V : a.D;  // loads per row
    int lg = 0;
    while ((1 << lg) < per && lg < 6) ++lg;
    const int64_t threads = rows << lg;
    hipLaunchKernelGGL((attn_bwd_pre_kernel<T>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, a, lg, vec);
  }
  dim3 gq((a.Lq + 63) / 64, a.B * a.H);
  bool done_dq = false, done_dkv = false;
  if constexpr (DP <= 64) {
    if (attn_fewq(a)) {
      if constexpr (sizeof(T) == 2 && DP == 32) hipLaunchKernelGGL((attn_bwd_dq_fewq_kernel<T, DP, 16>), dim3(a.B * a.H), dim3(1024), 0, st, a);
      else hipLaunchKernelGGL((attn_bwd_dq_fewq_kernel<T, DP>), dim3(a.B * a.H), dim3(256), 0, st, a);
      done_dq = true;
    }
    if (attn_fewk(a)) {
      if constexpr (sizeof(T) == 2 && DP == 32) hipLaunchKernelGGL((attn_bwd_dkv_fewk_kernel<T, DP, 8>), dim3(a.B * a.H), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bwd_dkv_fewk_kernel<T, DP>), dim3(a.B * a.H), dim3(256), 0, st, a);
      done_dkv = true;
    }
  }
  if constexpr (sizeof(T) == 2 && DP <= 64) {
    if (!done_dq && g_attn_win && a.Lk <= 16 && a.p_drop <= 0.f) {
      hipLaunchKernelGGL((attn_fewk_dq_kernel<DP>), dim3((a.Lq + 63) / 64, a.B * a.H), dim3(256), 0, st, a);
      done_dq = true;
    }
  }
  if (!done_dq) hipLaunchKernelGGL((attn_bwd_dq_kernel<T, DP>), gq, dim3(256), 0, st, a);
  constexpr int NW = AttnCfg<T>::NW_DKV;
  dim3 gk((a.Lk + NW * 16 - 1) / (NW * 16), a.B * a.H);
  if constexpr (sizeof(T) == 2 && DP <= 64) {
    if (!done_dkv && g_attn_win && a.Lq <= 16 && a.p_drop <= 0.f) {
      hipLaunchKernelGGL((attn_fewq_dkv_kernel<DP>), dim3((a.Lk + 63) / 64, a.B * a.H), dim3(256), 0, st, a);
      done_dkv = true;
    }
  }
  if (!done_dkv) hipLaunchKernelGGL((attn_bwd_dkv_kernel<T, DP>), gk, dim3(NW * 64), 0, st, a);
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}

template <typename T, bool FWD>
static int attn_dispatch(const AttnArgs& a, hipStream_t st) {
  if (a.D <= 32) return FWD ? attn_fwd_launch<T, 32>(a, st) : attn_bwd_launch<T, 32>(a, st);
  if (a.D <= 64) return FWD ? attn_fwd_launch<T, 64>(a, st) : attn_bwd_launch<T, 64>(a, st);
  if (a.D <= 96) return FWD ? attn_fwd_launch<T, 96>(a, st) : attn_bwd_launch<T, 96>(a, st);
  if (a.D <= 128) return FWD ? attn_fwd_launch<T, 128>(a, st) : attn_bwd_launch<T, 128>(a, st);
  if (a.D <= 256) return FWD ? attn_fwd_launch<T, 256>(a, st) : attn_bwd_launch<T, 256>(a, st);
  return (int)hipErrorInvalidValue;
}

// the flash kernels address their LDS-DMA operands with 32-bit element offsets from the
// (batch, head) base: rows x row stride must stay below 2^31 elements
static bool flash_span_ok(int64_t rows, int64_t stride) { return rows * (stride < 0 ? -stride : stride) < (1ll << 31); }

static bool attn_aligned(int dt, int D, const void* p, int64_t s1, int64_t s2, int64_t s3) {
  const int vec = dt == S2H_BF16 ? 8 : 4;
  return ((uintptr_t)p % 16 == 0) && D % vec == 0 && s1 % vec == 0 && s2 % vec == 0 && s3 % vec == 0;
}

extern "C" int s2h_attn_fwd(int dt, int B, int H, int Lq, int Lk, int D,
                            const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                            const void* k, int64_t skb, int64_t skh, int64_t skl,
                            const void* v, int64_t svb, int64_t svh, int64_t svl,
                            void* o, int64_t sob, int64_t soh, int64_t sol,
                            float* lse, float scale, float p_drop, uint64_t seed, uint64_t idx0, uint32_t* keep,
                            void* ws, int64_t ws_bytes, hipStream_t st) {
  if (B * H <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || D <= 0 || D > 256) return (int)hipErrorInvalidValue;
  if (!attn_aligned(dt, D, q, sqb, sqh, sql) || !attn_aligned(dt, D, k, skb, skh, skl) ||
      !attn_aligned(dt, D, v, svb, svh, svl))
    return (int)hipErrorInvalidValue;
  const bool flash = s2h_flash_eligible(dt, Lq, D) && attn_aligned(dt, D, o, sob, soh, sol) &&
                     flash_span_ok(Lk, skl) && flash_span_ok(Lk, svl);
  // a keep bitmap is written by the flash path only, for the head-dim-256 backward that reads it
  if (keep && p_drop > 0.f && (!flash || D != 256)) return (int)hipErrorInvalidValue;
  if (flash) {
    const int slot = s2h_prof_begin(st, 1, (int64_t)B * H, Lq, Lk, D, 2);
    const int rc = s2h_flash_fwd(B, H, Lq, Lk, D, q, sqb, sqh, sql, k, skb, skh, skl, v, svb, svh, svl, o, sob, soh,
                                 sol, lse, scale, p_drop, seed, idx0, keep, ws, ws_bytes, st);
    s2h_prof_end(slot, st);
    return rc;
  }
  AttnArgs a = {};
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.D = D;
  a.q = q; a.sqb = sqb; a.sqh = sqh; a.sql = sql;
  a.k = k; a.skb = skb; a.skh = skh; a.skl = skl;
  a.v = v; a.svb = svb; a.svh = svh; a.svl = svl;
  a.o = o; a.sob = sob; a.soh = soh; a.sol = sol;
  a.lse = lse; a.scale = scale; a.p_drop = p_drop; a.seed = seed; a.seed_off = s2h_rng_offset_ptr();
  a.idx0 = idx0;
  if (dt == S2H_BF16 && attn_win_ok(a, true) && attn_aligned(dt, D, o, sob, soh, sol)) return attn_win_launch<true>(a, st);
  return dt == S2H_BF16 ? attn_dispatch<bf16, true>(a, st) : attn_dispatch<float, true>(a, st);
}

extern "C" int s2h_attn_bwd(int dt, int B, int H, int Lq, int Lk, int D,
                            const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                            const void* k, int64_t skb, int64_t skh, int64_t skl,
                            const void* v, int64_t svb, int64_t svh, int64_t svl,
                            const void* o, int64_t sob, int64_t soh, int64_t sol,
                            const void* dout, int64_t sgb, int64_t sgh, int64_t sgl,
                            void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql,
                            void* dk, int64_t sdkb, int64_t sdkh, int64_t sdkl,
                            void* dv, int64_t sdvb, int64_t sdvh, int64_t sdvl,
                            const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                            uint64_t idx0, const uint32_t* keep, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (B * H <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || D <= 0 || D > 256) return (int)hipErrorInvalidValue;
  if (!attn_aligned(dt, D, q, sqb, sqh, sql) || !attn_aligned(dt, D, k, skb, skh, skl) ||
      !attn_aligned(dt, D, v, svb, svh, svl) || !attn_aligned(dt, D, dout, sgb, sgh, sgl))
    return (int)hipErrorInvalidValue;
  const bool flash = s2h_flash_bwd_eligible(dt, Lq, D) && attn_aligned(dt, D, o, sob, soh, sol) &&
                     attn_aligned(dt, D, dq, sdqb, sdqh, sdql) && attn_aligned(dt, D, dk, sdkb, sdkh, sdkl) &&
                     attn_aligned(dt, D, dv, sdvb, sdvh, sdvl) && flash_span_ok(Lk, skl) &&
                     flash_span_ok(Lk, svl) && flash_span_ok(Lq, sql) && flash_span_ok(Lq, sgl);
  if (keep && p_drop > 0.f && (!flash || D != 256)) return (int)hipErrorInvalidValue;
  if (flash) {
    const int slot = s2h_prof_begin(st, 2, (int64_t)B * H, Lq, Lk, D, 2);
    const int rc = s2h_flash_bwd(B, H, Lq, Lk, D, q, sqb, sqh, sql, k, skb, skh, skl, v, svb, svh, svl, o, sob, soh,
                                 sol, dout, sgb, sgh, sgl, dq, sdqb, sdqh, sdql, dk, sdkb, sdkh, sdkl, dv, sdvb, sdvh,
                                 sdvl, lse, di_ws, scale, p_drop, seed, idx0, keep, ws, ws_bytes, st);
    s2h_prof_end(slot, st);
    return rc;
  }
  AttnArgs a = {};
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.D = D;
  a.q = q; a.sqb = sqb; a.sqh = sqh; a.sql = sql;
  a.k = k; a.skb = skb; a.skh = skh; a.skl = skl;
  a.v = v; a.svb = svb; a.svh = svh; a.svl = svl;
  a.o = (void*)dout; a.sob = sgb; a.soh = sgh; a.sol = sgl;
  a.fo = o; a.sfb = sob; a.sfh = soh; a.sfl = sol;
  a.dq = dq; a.sdqb = sdqb; a.sdqh = sdqh; a.sdql = sdql;
  a.dk = dk; a.sdkb = sdkb; a.sdkh = sdkh; a.sdkl = sdkl;
  a.dv = dv; a.sdvb = sdvb; a.sdvh = sdvh; a.sdvl = sdvl;
  a.lse = (float*)lse; a.di = di_ws; a.scale = scale; a.p_drop = p_drop; a.seed = seed; a.seed_off = s2h_rng_offset_ptr();
  a.idx0 = idx0;
  if (dt == S2H_BF16 && attn_win_ok(a, false)) return attn_win_launch<false>(a, st);
  return dt == S2H_BF16 ? attn_dispatch<bf16, false>(a, st) : attn_dispatch<float, false>(a, st);
}
