// MOSI UTT-Fusion (BASELINE configs[4]; MML_Suite/models/msa/utt_fusion.py:25-200 with
// configs/mosi/centralised/utt_fusion_base_training.yaml): the recurrent LSTM encoders
// (models/msa/networks/lstm.py:8-67, nn.LSTM(batch_first) + "last" embedding), the TextCNN time-max
// pooling and its sparse weight gradient (models/msa/networks/textcnn.py:10-69), the global-norm
// gradient clip of train_step (utt_fusion.py:189, torch.nn.utils.clip_grad_norm_) and the padded
// sequence gather (data/mosi.py:202-232, pad_sequence).  The dense products around them (the LSTM
// input projection and weight gradients, the TextCNN convolutions, every Linear) run on the shared
// MFMA GEMM / implicit-GEMM conv kernels.
//
// Layout: sequences are TIME-MAJOR on the device — row (t, b) of a [T][B][F] tensor — so every
// step's rows are contiguous, the LSTM weight gradients are plain GEMMs over the T*B rows, and the
// text input is an HWNC tensor (H = T, W = 1, N = B, C = 768) for the LDS-staged conv kernel.
#include "common.h"

namespace {

TSPM_DEV float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// ------------------------------------------------------------------------------------------------
// LSTM forward: one workgroup per RB batch rows runs all T steps; thread j (of 4H) owns gate column
// j and keeps row j of W_hh in registers; h_{t-1} is broadcast from LDS.  ATen's LSTMCell order:
// gates = (h W_hh^T + b_hh) + (x W_ih^T + b_ih); i,f,o = sigmoid, g = tanh; c = f*c + i*g;
// h = o * tanh(c).  Saved for the backward: activated gates, c_t, h_t.
// ------------------------------------------------------------------------------------------------
struct LstmFwdDesc {
  int B, T;
  const float* xg;   // [T][B][4H]: x W_ih^T + b_ih
  const float* whh;  // [4H][H]
  const float* bhh;  // [4H] or null
  float* gates;      // [T][B][4H] activated i, f, g, o
  float* cs;         // [T][B][H]
  float* hs;         // [T+1][B][H], hs[0] = 0
  float* hout;       // h_T rows (embd "last") or max_t h_t (embd "maxpool"), stride ldh
  int ldh;
  uint8_t* arg;      // embd "maxpool": [B][H] time index of the maximum (F.max_pool1d), else null
};

template <int H, int RB>
TSPM_DEV void lstm_fwd_body(const LstmFwdDesc& d, int chunk) {
  constexpr int G = 4 * H;
  __shared__ __attribute__((aligned(16))) float hsh[RB][H];
  __shared__ float gsh[RB][G];
  const int j = threadIdx.x;
  const int b0 = chunk * RB;
  const int B = d.B, T = d.T;
  float w[H];
#pragma unroll
  for (int k = 0; k < H; k += 4) {
    const f32x4 v = ld4(d.whh + (long long)j * H + k);
    w[k] = v[0]; w[k + 1] = v[1]; w[k + 2] = v[2]; w[k + 3] = v[3];
  }
  const float bh = d.bhh ? d.bhh[j] : 0.f;
  // an odd batch leaves the last workgroup one row short: that ghost row reads the last real row's inputs
  // (clamped index) and writes nothing
  const int cr = j / H, cu = j - (j / H) * H;
  const bool cell = j < RB * H && b0 + cr < B;
  float c = 0.f, h = 0.f;
  float mx = -INFINITY;  // embd "maxpool": running max over t of h_t and its first index (NaN wins, as
  int am = 0;            // max_pool2d_with_indices: val > max || isnan(val))
  if (j < RB * H) hsh[cr][cu] = 0.f;
  if (cell) d.hs[(long long)(b0 + cr) * H + cu] = 0.f;
  const bool sig = j < 2 * H || j >= 3 * H;
  int rowc[RB];  // clamped row of each of the workgroup's rows
#pragma unroll
  for (int r = 0; r < RB; ++r) rowc[r] = min(b0 + r, B - 1);
  float xn[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) xn[r] = d.xg[(long long)rowc[r] * G + j];
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float xc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) xc[r] = xn[r];
    if (t + 1 < T) {
#pragma unroll
      for (int r = 0; r < RB; ++r) xn[r] = d.xg[((long long)(t + 1) * B + rowc[r]) * G + j];
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      // four interleaved partial sums (k mod 4): a 16-deep dependent FMA chain instead of 64
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < H; k += 4) {
        const f32x4 hv = *reinterpret_cast<const f32x4*>(&hsh[r][k]);
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] = fmaf(hv[u], w[k + u], a4[u]);
      }
      const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      const float pre = (acc + bh) + xc[r];
      const float a = sig ? sigmoidf_(pre) : tanhf(pre);
      gsh[r][j] = a;
      if (b0 + r < B) d.gates[((long long)t * B + b0 + r) * G + j] = a;
    }
    __syncthreads();
    if (j < RB * H) {
      const float ig = gsh[cr][cu], fg = gsh[cr][H + cu], gg = gsh[cr][2 * H + cu], og = gsh[cr][3 * H + cu];
      c = fg * c + ig * gg;
      h = og * tanhf(c);
      hsh[cr][cu] = h;
    }
    if (cell) {
      const long long o = ((long long)t * B + b0 + cr) * H + cu;
      d.cs[o] = c;
      d.hs[o + (long long)B * H] = h;
      if (d.arg && (h > mx || h != h)) {
        mx = h;
        am = t;
      }
    }
    __syncthreads();
  }
  if (cell) {
    d.hout[(long long)(b0 + cr) * d.ldh + cu] = d.arg ? mx : h;
    if (d.arg) d.arg[(long long)(b0 + cr) * H + cu] = (uint8_t)am;
  }
}

template <int H, int RB>
__global__ __launch_bounds__(4 * H) void k_lstm_fwd(LstmFwdDesc d0, LstmFwdDesc d1, int nb0) {
  if ((int)blockIdx.x < nb0)
    lstm_fwd_body<H, RB>(d0, blockIdx.x);
  else
    lstm_fwd_body<H, RB>(d1, blockIdx.x - nb0);
}

// ------------------------------------------------------------------------------------------------
// LSTM backward through time: thread (q, k) = (gate quarter, hidden unit) keeps column k of the
// quarter-q rows of W_hh in registers for dh_{t-1} = dgates_t @ W_hh (4 partial sums combined in
// fixed order through LDS); threads (r, u) carry dc and form the pre-activation gate gradients
// (written time-major for the weight-gradient GEMMs that follow).
// ------------------------------------------------------------------------------------------------
struct LstmBwdDesc {
  int B, T;
  const float* whh;    // [4H][H]
  const float* gates;  // [T][B][4H]
  const float* cs;     // [T][B][H]
  const float* dh;     // gradient of the embedding rows (h_T, or max_t h_t at arg), stride lddh
  int lddh;
  float* dgates;       // [T][B][4H] out
  const uint8_t* arg;  // embd "maxpool": [B][H] time index that received the embedding (null: T-1)
};

template <int H, int RB>
TSPM_DEV void lstm_bwd_body(const LstmBwdDesc& d, int chunk) {
  constexpr int G = 4 * H;
  __shared__ __attribute__((aligned(16))) float dgs[RB][G];
  __shared__ float part[4][RB][H];
  const int tid = threadIdx.x;
  const int q = tid / H, k = tid - (tid / H) * H;
  const int b0 = chunk * RB;
  const int B = d.B, T = d.T;
  float wc[H];
#pragma unroll
  for (int jj = 0; jj < H; ++jj) wc[jj] = d.whh[(long long)(q * H + jj) * H + k];
  const int cr = tid / H, cu = tid - (tid / H) * H;
  const bool cell = tid < RB * H && b0 + cr < B;  // a ghost row (odd batch) computes zeros, writes nothing
  float dc = 0.f, dh = 0.f, gin = 0.f;
  int am = T - 1;  // the step whose h received the embedding gradient
  if (cell) {
    gin = d.dh[(long long)(b0 + cr) * d.lddh + cu];
    if (d.arg) am = d.arg[(long long)(b0 + cr) * H + cu];
  }
  if (tid < RB * H && !cell) {
    dgs[cr][cu] = 0.f; dgs[cr][H + cu] = 0.f; dgs[cr][2 * H + cu] = 0.f; dgs[cr][3 * H + cu] = 0.f;
  }
  for (int t = T - 1; t >= 0; --t) {
    if (cell) {
      if (t < T - 1) {
        dh = ((part[0][cr][cu] + part[1][cr][cu]) + part[2][cr][cu]) + part[3][cr][cu];
        if (t == am) dh += gin;  // max-pooled embedding: its gradient joins the recurrent one at the argmax
      } else {
        dh = am == T - 1 ? gin : 0.f;
      }
      const long long go = ((long long)t * B + b0 + cr) * G + cu;
      const float ig = d.gates[go], fg = d.gates[go + H], gg = d.gates[go + 2 * H], og = d.gates[go + 3 * H];
      const long long co = ((long long)t * B + b0 + cr) * H + cu;
      const float c = d.cs[co];
      const float cp = t > 0 ? d.cs[co - (long long)B * H] : 0.f;
      const float tc = tanhf(c);
      const float dog = dh * tc;
      const float dcc = dc + dh * og * (1.f - tc * tc);
      const float dig = dcc * gg, dgg = dcc * ig, dfg = dcc * cp;
      dc = dcc * fg;
      const float ai = dig * ig * (1.f - ig), af = dfg * fg * (1.f - fg);
      const float ag = dgg * (1.f - gg * gg), ao = dog * og * (1.f - og);
      dgs[cr][cu] = ai; dgs[cr][H + cu] = af; dgs[cr][2 * H + cu] = ag; dgs[cr][3 * H + cu] = ao;
      d.dgates[go] = ai; d.dgates[go + H] = af; d.dgates[go + 2 * H] = ag; d.dgates[go + 3 * H] = ao;
    }
    __syncthreads();
    if (t > 0) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        float a4[4] = {0.f, 0.f, 0.f, 0.f};  // interleaved partial sums, as in the forward
#pragma unroll
        for (int jj = 0; jj < H; jj += 4) {
          const f32x4 dv = *reinterpret_cast<const f32x4*>(&dgs[r][q * H + jj]);
#pragma unroll
          for (int u = 0; u < 4; ++u) a4[u] = fmaf(dv[u], wc[jj + u], a4[u]);
        }
        part[q][r][k] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
    }
    __syncthreads();
  }
}

template <int H, int RB>
__global__ __launch_bounds__(4 * H) void k_lstm_bwd(LstmBwdDesc d0, LstmBwdDesc d1, int nb0) {
  if ((int)blockIdx.x < nb0)
    lstm_bwd_body<H, RB>(d0, blockIdx.x);
  else
    lstm_bwd_body<H, RB>(d1, blockIdx.x - nb0);
}

// ------------------------------------------------------------------------------------------------
// TextCNN pooling: conv_i [Tout_i][B][C] (+ bias) -> ReLU -> max over time (first maximum, as
// F.max_pool1d) for every (b, conv i, channel); the result (and its dropout, textcnn.py:66) goes to
// the embedding Linear's input.  The argmax time index and the pooled value are kept for the backward.
// ------------------------------------------------------------------------------------------------
struct PoolSet {
  const float* y[4];
  const float* bias[4];
  int kh[4];
};

__global__ __launch_bounds__(256) void k_textcnn_pool(int B, int T, int nconv, int C, PoolSet ps,
                                                      const uint8_t* __restrict__ keep, float scale,
                                                      float* __restrict__ pre, uint8_t* __restrict__ arg,
                                                      float* __restrict__ out, int ldo) {
  const int nc = nconv * C;
  const long long total = (long long)B * nc;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int b = (int)(e / nc), ci = (int)(e - (long long)b * nc);
    const int i = ci / C, c = ci - i * C;
    const int tout = T - ps.kh[i] + 1;
    const float* y = ps.y[i];
    const float bv = ps.bias[i] ? ps.bias[i][c] : 0.f;
    float best = -1.f;
    int bi = 0;
    for (int t = 0; t < tout; ++t) {
      float v = y[((long long)t * B + b) * C + c] + bv;
      v = v > 0.f ? v : (v != v ? v : 0.f);  // ReLU (NaN propagates)
      if (v > best || v != v) { best = v; bi = t; }
    }
    pre[e] = best;
    arg[e] = (uint8_t)bi;
    out[(long long)b * ldo + ci] = keep ? best * (keep[e] ? scale : 0.f) : best;
  }
}

// grad of the pooled features: through the dropout (keep * scale) and the ReLU at the argmax.
__global__ __launch_bounds__(256) void k_textcnn_pool_grad(long long total, int nc, const float* __restrict__ dout,
                                                           int ldd, const uint8_t* __restrict__ keep, float scale,
                                                           const float* __restrict__ pre, float* __restrict__ g) {
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long b = e / nc, ci = e - b * nc;
    float v = dout[b * ldd + ci];
    if (keep) v = v * (keep[e] ? scale : 0.f);
    g[e] = pre[e] > 0.f ? v : 0.f;
  }
}

// Sparse weight gradient of conv i: dW[c][dt][f] = sum_b g[b][c] x[arg[b][c] + dt][b][f] (only the
// argmax position of each (b, c) carries gradient after the time-max), db[c] = sum_b g[b][c].
// One workgroup per (conv, channel); threads over f; the kh rows of a window accumulate in registers.
struct WgradSet {
  float* dw[4];
  float* db[4];
  int kh[4];
};

template <int KMAX, int FPT>
__global__ __launch_bounds__(256) void k_textcnn_wgrad(int B, int F, int C, WgradSet ws, const float* __restrict__ x,
                                                       const float* __restrict__ g, const uint8_t* __restrict__ arg,
                                                       int nc) {
  const int i = blockIdx.x / C, c = blockIdx.x - (blockIdx.x / C) * C;
  const int kh = ws.kh[i];
  const int ci = i * C + c;
  float acc[KMAX][FPT];
#pragma unroll
  for (int dt = 0; dt < KMAX; ++dt)
#pragma unroll
    for (int u = 0; u < FPT; ++u) acc[dt][u] = 0.f;
  for (int b = 0; b < B; ++b) {
    const float gv = g[(long long)b * nc + ci];
    if (gv == 0.f) continue;  // workgroup-uniform
    const int t0 = arg[(long long)b * nc + ci];
#pragma unroll
    for (int dt = 0; dt < KMAX; ++dt) {
      if (dt >= kh) break;
      const float* row = x + ((long long)(t0 + dt) * B + b) * F;
#pragma unroll
      for (int u = 0; u < FPT; ++u) {
        const int f = threadIdx.x + 256 * u;
        if (f < F) acc[dt][u] = fmaf(gv, row[f], acc[dt][u]);
      }
    }
  }
  float* dw = ws.dw[i] + (long long)c * kh * F;
#pragma unroll
  for (int dt = 0; dt < KMAX; ++dt) {
    if (dt >= kh) break;
#pragma unroll
    for (int u = 0; u < FPT; ++u) {
      const int f = threadIdx.x + 256 * u;
      if (f < F) dw[(long long)dt * F + f] = acc[dt][u];
    }
  }
  if (threadIdx.x == 0 && ws.db[i]) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += g[(long long)b * nc + ci];
    ws.db[i][c] = s;
  }
}

// Same gradient, organised for HBM reuse (C = 128 channels): one workgroup per (conv, 8-float slice of
// the 768 features).  Each step stages NBS batch rows' [T][8] input slices, the g and argmax of those
// rows in LDS; thread (c = tid / 2, 4 features) accumulates dW[c][0..kh)[4] over b in ascending order —
// the same fmaf sequence as k_textcnn_wgrad, so the two are bitwise identical — while the input is read
// from HBM once per conv (T*B*F*4 bytes) instead of once per (channel, batch row) window.
constexpr int kWgFB = 8;    // features per workgroup
constexpr int kWgNBS = 8;   // batch rows staged per LDS round
constexpr int kWgC = 128;   // channels (2 threads each)

template <int KMAX>
__global__ __launch_bounds__(256) void k_textcnn_wgrad_slab(int B, int T, int F, WgradSet ws, const float* __restrict__ x,
                                                            const float* __restrict__ g,
                                                            const uint8_t* __restrict__ arg, int nc, int nfb) {
  __shared__ float4 xs[kWgNBS][256][kWgFB / 4];  // [row][t][8 floats]; T <= 256
  __shared__ float gs[kWgNBS][kWgC];
  __shared__ int as_[kWgNBS][kWgC];
  const int i = blockIdx.x / nfb, fb = blockIdx.x - (blockIdx.x / nfb) * nfb;
  const int kh = ws.kh[i], f0 = fb * kWgFB;
  const int tid = threadIdx.x, c = tid >> 1, half = tid & 1;
  const int ci = i * kWgC + c;
  float4 acc[KMAX];
#pragma unroll
  for (int dt = 0; dt < KMAX; ++dt) acc[dt] = make_float4(0.f, 0.f, 0.f, 0.f);
  float dbs = 0.f;
  for (int b0 = 0; b0 < B; b0 += kWgNBS) {
    const int nb = B - b0 < kWgNBS ? B - b0 : kWgNBS;
    __syncthreads();
    for (int e = tid; e < nb * T * 2; e += 256) {  // 2 float4 per (row, t)
      const int q = e & 1, rt = e >> 1, r = rt / T, t = rt - r * T;
      xs[r][t][q] = *reinterpret_cast<const float4*>(x + ((long long)t * B + b0 + r) * F + f0 + 4 * q);
    }
    for (int e = tid; e < nb * kWgC; e += 256) {
      const int r = e / kWgC, cc = e - r * kWgC;
      gs[r][cc] = g[(long long)(b0 + r) * nc + i * kWgC + cc];
      as_[r][cc] = arg[(long long)(b0 + r) * nc + i * kWgC + cc];
    }
    __syncthreads();
    for (int r = 0; r < nb; ++r) {
      const float gv = gs[r][c];
      if (half == 0) dbs += gv;
      if (gv == 0.f) continue;
      const int t0 = as_[r][c];
#pragma unroll
      for (int dt = 0; dt < KMAX; ++dt) {
        if (dt >= kh) break;
        const float4 v = xs[r][t0 + dt][half];
        acc[dt].x = fmaf(gv, v.x, acc[dt].x);
        acc[dt].y = fmaf(gv, v.y, acc[dt].y);
        acc[dt].z = fmaf(gv, v.z, acc[dt].z);
        acc[dt].w = fmaf(gv, v.w, acc[dt].w);
      }
    }
  }
  float* dw = ws.dw[i] + (long long)c * kh * F;
#pragma unroll
  for (int dt = 0; dt < KMAX; ++dt) {
    if (dt >= kh) break;
    *reinterpret_cast<float4*>(dw + (long long)dt * F + f0 + 4 * half) = acc[dt];
  }
  if (fb == 0 && half == 0 && ws.db[i]) ws.db[i][c] = dbs;
  (void)ci;
}

// ------------------------------------------------------------------------------------------------
// Global-norm gradient clip (torch.nn.utils.clip_grad_norm_, norm 2): sum of squares of
// (grad * grad_scale) in double per workgroup, then one workgroup sums the partials in index order
// and writes coef = min(1, max_norm / (total_norm + 1e-6)) for the Adam launch that follows.
// ------------------------------------------------------------------------------------------------
constexpr int kClipBlocks = 512;

__global__ __launch_bounds__(256) void k_sumsq(long long count, const float* __restrict__ g, float gs,
                                               double* __restrict__ partial) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < count; i += (long long)gridDim.x * 256) {
    const double v = (double)(g[i] * gs);
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// one workgroup: strided partial sums then a fixed-order LDS tree (deterministic; all loads in flight
// together instead of one thread's dependent chain)
__global__ __launch_bounds__(256) void k_clip_coef(int nparts, const double* __restrict__ partial, float max_norm,
                                                   float* __restrict__ coef, float* __restrict__ norm_out) {
  __shared__ double red[256];
  double a = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) a += partial[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double s = red[0];
  const float total = (float)sqrt(s);
  const float cf = max_norm / (total + 1e-6f);
  coef[0] = cf < 1.f ? cf : 1.f;
  if (norm_out) norm_out[0] = total;
}

// ------------------------------------------------------------------------------------------------
// Padded sequence gather (pad_sequence(batch_first) of data/mosi.py:225-230 + the step's .to(device)):
// out[t][b][:] (time-major, strides st / sb) = row offset[idx_b] + t of the ragged corpus if
// t < length[idx_b], else 0; times the per-row modality mask; labels gathered alongside.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_seq_gather(int nb, const int64_t* __restrict__ index, long long nsamp,
                                                    const float* __restrict__ data, const int64_t* __restrict__ offs,
                                                    const int32_t* __restrict__ lens, int F, int Tpad,
                                                    float* __restrict__ out, long long st, long long sb,
                                                    const float* __restrict__ mask, const int64_t* __restrict__ lab_in,
                                                    int64_t* __restrict__ lab_out) {
  const long long total = (long long)Tpad * nb * F;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int f = (int)(e % F);
    const long long tb = e / F;
    const int b = (int)(tb % nb), t = (int)(tb / nb);
    const long long s = index[b];
    float v;
    if (s < 0 || s >= nsamp) {
      v = __builtin_nanf("");
    } else {
      v = t < lens[s] ? data[(offs[s] + t) * (long long)F + f] : 0.f;
      if (mask) v = v * mask[b];
    }
    out[(long long)t * st + (long long)b * sb + f] = v;
    if (lab_out && t == 0 && f == 0) lab_out[b] = (s < 0 || s >= nsamp) ? -1 : lab_in[s];
  }
}

int grid_for(long long work) {
  long long b = cdiv64(work, 256);
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

template <int H, int RB>
int launch_lstm_fwd(const LstmFwdDesc& a, const LstmFwdDesc* b, hipStream_t st) {
  const int na = (a.B + RB - 1) / RB, nbb = b ? (b->B + RB - 1) / RB : 0;
  hipLaunchKernelGGL((k_lstm_fwd<H, RB>), dim3(na + nbb), dim3(4 * H), 0, st, a, b ? *b : a, na);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

template <int H, int RB>
int launch_lstm_bwd(const LstmBwdDesc& a, const LstmBwdDesc* b, hipStream_t st) {
  const int na = (a.B + RB - 1) / RB, nbb = b ? (b->B + RB - 1) / RB : 0;
  hipLaunchKernelGGL((k_lstm_bwd<H, RB>), dim3(na + nbb), dim3(4 * H), 0, st, a, b ? *b : a, na);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

constexpr int kLstmRB = 2;  // batch rows per workgroup (B = 128: 64 workgroups per LSTM)

bool lstm_ok(int B, int T, int H, const void* p0, const void* p1, const void* p2, const void* p3) {
  return B > 0 && T > 0 && H == 64 && p0 && p1 && p2 && p3;
}

}  // namespace

extern "C" int tspm_lstm_fwd(int32_t count, const tspm_lstm_fwd_desc* descs, tspm_stream_t stream) {
  if (count < 1 || count > 2 || !descs) return TSPM_ERR_INVALID;
  LstmFwdDesc d[2];
  for (int i = 0; i < count; ++i) {
    const tspm_lstm_fwd_desc& s = descs[i];
    if (!lstm_ok(s.batch, s.steps, s.hidden, s.xg, s.w_hh, s.gates, s.cs) || !s.hs || !s.h_out || s.ld_out < s.hidden)
      return TSPM_ERR_INVALID;
    if (reinterpret_cast<uintptr_t>(s.w_hh) & 15) return TSPM_ERR_INVALID;
    if (s.steps > 256 && s.argmax) return TSPM_ERR_INVALID;  // uint8 time index
    d[i] = LstmFwdDesc{s.batch, s.steps, s.xg, s.w_hh, s.b_hh, s.gates, s.cs, s.hs, s.h_out, s.ld_out, s.argmax};
  }
  return launch_lstm_fwd<64, kLstmRB>(d[0], count > 1 ? &d[1] : nullptr, static_cast<hipStream_t>(stream));
}

extern "C" int tspm_lstm_bwd(int32_t count, const tspm_lstm_bwd_desc* descs, tspm_stream_t stream) {
  if (count < 1 || count > 2 || !descs) return TSPM_ERR_INVALID;
  LstmBwdDesc d[2];
  for (int i = 0; i < count; ++i) {
    const tspm_lstm_bwd_desc& s = descs[i];
    if (!lstm_ok(s.batch, s.steps, s.hidden, s.w_hh, s.gates, s.cs, s.dh) || !s.dgates || s.ld_dh < s.hidden)
      return TSPM_ERR_INVALID;
    if (s.steps > 256 && s.argmax) return TSPM_ERR_INVALID;
    d[i] = LstmBwdDesc{s.batch, s.steps, s.w_hh, s.gates, s.cs, s.dh, s.ld_dh, s.dgates, s.argmax};
  }
  return launch_lstm_bwd<64, kLstmRB>(d[0], count > 1 ? &d[1] : nullptr, static_cast<hipStream_t>(stream));
}

extern "C" int tspm_textcnn_pool_fwd(int32_t batch, int32_t steps, int32_t nconv, const int32_t* heights,
                                     int32_t channels, const float* const* conv_out, const float* const* bias,
                                     const uint8_t* keep, float keep_scale, float* pooled, uint8_t* argmax,
                                     float* out, int32_t ld_out, tspm_stream_t stream) {
  if (batch <= 0 || steps <= 0 || nconv < 1 || nconv > 4 || !heights || channels <= 0 || !conv_out || !pooled ||
      !argmax || !out || ld_out < nconv * channels || steps > 256)
    return TSPM_ERR_INVALID;
  PoolSet ps{};
  for (int i = 0; i < nconv; ++i) {
    if (heights[i] < 1 || heights[i] > steps || !conv_out[i]) return TSPM_ERR_INVALID;
    ps.y[i] = conv_out[i];
    ps.bias[i] = bias ? bias[i] : nullptr;
    ps.kh[i] = heights[i];
  }
  hipLaunchKernelGGL(k_textcnn_pool, dim3(grid_for((long long)batch * nconv * channels)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), batch, steps, nconv, channels, ps, keep, keep_scale, pooled,
                     argmax, out, ld_out);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_textcnn_bwd(int32_t batch, int32_t steps, int32_t feat, int32_t nconv, const int32_t* heights,
                                int32_t channels, const float* x, const float* dout, int32_t ld_dout,
                                const uint8_t* keep, float keep_scale, const float* pooled, const uint8_t* argmax,
                                float* const* dw, float* const* db, float* g_work, tspm_stream_t stream) {
  if (batch <= 0 || steps <= 0 || feat <= 0 || feat > 1024 || nconv < 1 || nconv > 4 || !heights || channels <= 0 ||
      !x || !dout || !pooled || !argmax || !dw || !g_work || ld_dout < nconv * channels)
    return TSPM_ERR_INVALID;
  WgradSet ws{};
  for (int i = 0; i < nconv; ++i) {
    if (heights[i] < 1 || heights[i] > 5 || heights[i] > steps || !dw[i]) return TSPM_ERR_INVALID;
    ws.dw[i] = dw[i];
    ws.db[i] = db ? db[i] : nullptr;
    ws.kh[i] = heights[i];
  }
  const int nc = nconv * channels;
  const long long total = (long long)batch * nc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_textcnn_pool_grad, dim3(grid_for(total)), dim3(256), 0, st, total, nc, dout, ld_dout, keep,
                     keep_scale, pooled, g_work);
  TSPM_LAUNCH_CHECK();
  const bool slab = channels == kWgC && feat % kWgFB == 0 && steps <= 256 &&
                    (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (slab) {
    for (int i = 0; i < nconv; ++i)
      if (reinterpret_cast<uintptr_t>(dw[i]) & 15) return TSPM_ERR_INVALID;
    const int nfb = feat / kWgFB;
    hipLaunchKernelGGL((k_textcnn_wgrad_slab<5>), dim3(nconv * nfb), dim3(256), 0, st, batch, steps, feat, ws, x, g_work,
                       argmax, nc, nfb);
  } else {
    hipLaunchKernelGGL((k_textcnn_wgrad<5, 4>), dim3(nc), dim3(256), 0, st, batch, feat, channels, ws, x, g_work,
                       argmax, nc);
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" size_t tspm_grad_clip_workspace(void) { return (size_t)kClipBlocks * sizeof(double); }

extern "C" int tspm_grad_clip_coef(int64_t count, const float* grad, float grad_scale, float max_norm, float* coef,
                                   float* total_norm, void* workspace, size_t workspace_bytes, tspm_stream_t stream) {
  if (count <= 0 || !grad || !coef || !workspace || workspace_bytes < tspm_grad_clip_workspace() || !(max_norm > 0.f))
    return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_sumsq, dim3(kClipBlocks), dim3(256), 0, st, (long long)count, grad, grad_scale, part);
  TSPM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_clip_coef, dim3(1), dim3(256), 0, st, kClipBlocks, part, max_norm, coef, total_norm);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_seq_gather(int32_t count, const int64_t* index, int64_t n_samples, const float* data,
                               const int64_t* offsets, const int32_t* lengths, int32_t feat, int32_t steps_pad,
                               float* out, int64_t stride_t, int64_t stride_b, const float* row_mask,
                               const int64_t* labels, int64_t* labels_out, tspm_stream_t stream) {
  if (count <= 0 || !index || n_samples <= 0 || !data || !offsets || !lengths || feat <= 0 || steps_pad <= 0 || !out)
    return TSPM_ERR_INVALID;
  if ((labels == nullptr) != (labels_out == nullptr)) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_seq_gather, dim3(grid_for((long long)steps_pad * count * feat)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), count, index, (long long)n_samples, data, offsets, lengths, feat,
                     steps_pad, out, (long long)stride_t, (long long)stride_b, row_mask, labels, labels_out);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
