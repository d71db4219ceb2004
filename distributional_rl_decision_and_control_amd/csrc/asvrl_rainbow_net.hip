// asvrl_rainbow_net.hip -- Rainbow_Policy's forward pass and dueling C51 head in one launch on gfx950
// (rfarl/rfarl/policy/Rainbow_model.py:97-139, agent.py:308-324 act_rainbow, agent.py:605-612 the
// double-Q target of train_Rainbow).
//
// The network per row: f = [relu(self_encoder(s_self)) | masked relu(object_encoder(s_obj))] (256),
//   value     hv1 = relu(Wv1 f + bv1), hv2 = relu(Wv2 hv1 + bv2), v = Wvo hv2 + bvo          (51)
//   advantage ha1 = relu(Wa1 f + ba1), ha2 = relu(Wa2 ha1 + ba2), a = Wao ha2 + bao      (25 x 51)
//   q[k] = v + a[k] - mean_k a[k], p[k] = softmax over atoms, Q[k] = sum p[k] z.
// The NoisyLinear weights enter composed (W = mu + sigma eps, asvrl_noisy_compose / _reset).
//
// One workgroup of 4 waves per 32-row tile; the waves split every layer's output features and exchange
// the activations through LDS in chained position order (asvrl_lds.h), so a launch of B rows runs
// 4 B / 32 waves and the weight fragments are read from L2 once per tile. mean_k a[k] is one more
// 51-row layer whose weights are the action-mean of output_layer_a's rows (packed by
// asvrl_rainbow_pack): the head then needs each action's 51 logits only once, in registers -- the
// 25 x 51 advantage logits never leave the wave that computes them. Waves own actions w, w+4, ...;
// the argmax over actions is reduced across waves through LDS (first maximum, as torch.argmax).
//
// Modes: ACT     argmax_k Q[k] with epsilon-greedy on the device step counter (act_out, f64)
//        ARGMAX  argmax_k Q[k] (act_idx; the online net on s_{t+n})
//        PICK    p[a*] for a* = act_idx[row] (the target net on s_{t+n}, p_out [N][51])
#include "asvrl_common.h"
#include "asvrl_mfma.h"
#include "asvrl_lds.h"

namespace asvrl {
namespace {

constexpr int kAtoms = 51, kActs = 25, kAP = 64, kEnc = 256, kHid = 128, kObsK = 32;
constexpr int kSelfF = 56, kObjF = 40, kSelfIn = 7, kObjIn = 5, kObjN = 5;
constexpr int kNW = 4;
enum { RB_ACT = 0, RB_ARGMAX = 1, RB_PICK = 2 };

struct RbArgs {
  AsvRainbowImg w;
  AsvRainbowNetIO io;
};

struct RbLds {
  elem_t x0[32 * kEnc];            // f; then hv2 | ha2 (x0 is dead after the first hidden layers)
  elem_t h1[2][32 * kHid];         // hv1, ha1; then v and the action-mean logits (f32)
  float z[kAP];
  float best_q[kNW][32];
  int best_k[kNW][32];
};
static_assert(2 * 32 * kHid * sizeof(elem_t) >= 2 * 32 * kAP * sizeof(float), "v / mean logits fit over h1");

// object index of encoder feature m (>= 56)
__device__ __forceinline__ int obj_of(int m) { return (m - kSelfF) / kObjF; }

template <int MODE>
__global__ __launch_bounds__(kNW * 64) void rainbow_net_kernel(RbArgs a) {
  __shared__ __attribute__((aligned(16))) RbLds L;
  const AsvRainbowNetIO& io = a.io;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int row0 = blockIdx.x * 32;
  const int row = row0 + r;
  const bool valid = row < io.N;
  const int64_t rr = valid ? row : io.N - 1;
  if (threadIdx.x < kAP) L.z[threadIdx.x] = threadIdx.x < kAtoms ? io.support[threadIdx.x] : 0.f;

  // ---------------- encoders (wave w: features 64w .. 64w + 63) -> f in x0
  {
    const float* xr = io.x + rr * io.ldx;
    frag8 bx[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(xr + ks * 16 + 8 * h);
      const f32x4 v = *reinterpret_cast<const f32x4*>(xr + ks * 16 + 8 * h + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bx[ks][j] = (elem_t)u[j];
        bx[ks][4 + j] = (elem_t)v[j];
      }
    }
    float mk[kObjN];
#pragma unroll
    for (int o = 0; o < kObjN; ++o) mk[o] = xr[32 + o];
    const frag8* ENC = reinterpret_cast<const frag8*>(a.w.enc);
    const RowA<kEnc> RA(r, h);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int mb = 2 * w + q;
      f32x16 acc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) acc = mfma(ENC[(mb * 2 + ks) * 64 + lane], bx[ks], acc);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        frag8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = feat(mb, 8 * s + i, h);
          const int ob = m < kSelfF ? -1 : obj_of(m);   // select chain: no dynamic register index
          const float mo = ob == 0 ? mk[0] : ob == 1 ? mk[1] : ob == 2 ? mk[2] : ob == 3 ? mk[3] : mk[4];
          const float keep = ob < 0 ? 1.f : (mo < 0.5f ? 0.f : 1.f);   // masked_fill(mask < 0.5, 0)
          o[i] = (elem_t)(relu(acc[8 * s + i] + a.w.b_enc[m]) * keep);
        }
        rows(L.x0, RA, 0, 2 * mb + s, o);
      }
    }
  }
  __syncthreads();

  // ---------------- hv1, ha1 (wave w: block w of each)
  {
    const frag8* V1 = reinterpret_cast<const frag8*>(a.w.v1);
    const frag8* A1 = reinterpret_cast<const frag8*>(a.w.a1);
    const RowA<kEnc> RX(r, h);
    const RowA<kHid> RH(r, h);
    f32x16 av = acc_init(a.w.b_v1p, w * 32, h), aa = acc_init(a.w.b_a1p, w * 32, h);
#pragma unroll
    for (int ks = 0; ks < kEnc / 16; ++ks) {
      const frag8 b = rowf(L.x0, RX, 0, ks);
      av = mfma(V1[(w * 16 + ks) * 64 + lane], b, av);
      aa = mfma(A1[(w * 16 + ks) * 64 + lane], b, aa);
    }
    if constexpr (!kBiasFirst) {
      av += bias_init(a.w.b_v1p, w * 32, h);
      aa += bias_init(a.w.b_a1p, w * 32, h);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      frag8 ov, oa;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ov[i] = (elem_t)relu(av[8 * s + i]);
        oa[i] = (elem_t)relu(aa[8 * s + i]);
      }
      rows(L.h1[0], RH, 0, 2 * w + s, ov);
      rows(L.h1[1], RH, 0, 2 * w + s, oa);
    }
  }
  __syncthreads();

  // ---------------- hv2, ha2 into x0's space
  elem_t* const hv2 = L.x0;
  elem_t* const ha2 = L.x0 + 32 * kHid;
  {
    const frag8* V2 = reinterpret_cast<const frag8*>(a.w.v2);
    const frag8* A2 = reinterpret_cast<const frag8*>(a.w.a2);
    const RowA<kHid> RH(r, h);
    f32x16 av = acc_init(a.w.b_v2p, w * 32, h), aa = acc_init(a.w.b_a2p, w * 32, h);
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) {
      av = mfma(V2[(w * 8 + ks) * 64 + lane], rowf(L.h1[0], RH, 0, ks), av);
      aa = mfma(A2[(w * 8 + ks) * 64 + lane], rowf(L.h1[1], RH, 0, ks), aa);
    }
    if constexpr (!kBiasFirst) {
      av += bias_init(a.w.b_v2p, w * 32, h);
      aa += bias_init(a.w.b_a2p, w * 32, h);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      frag8 ov, oa;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ov[i] = (elem_t)relu(av[8 * s + i]);
        oa[i] = (elem_t)relu(aa[8 * s + i]);
      }
      rows(hv2, RH, 0, 2 * w + s, ov);
      rows(ha2, RH, 0, 2 * w + s, oa);
    }
  }
  __syncthreads();

  // ---------------- v (waves 0, 1: atom blocks 0, 1) and the action-mean logits (waves 2, 3), f32 in
  // h1's space (last read by layer 2, behind the barrier), row-major [32][64] in natural atom order
  float* const vl = reinterpret_cast<float*>(&L.h1[0][0]);
  float* const ml = vl + 32 * kAP;
  {
    const bool val = w < 2;
    const int blk = w & 1;
    const frag8* W = reinterpret_cast<const frag8*>(val ? a.w.vo : a.w.mo);
    const float* bias = val ? a.w.b_vop : a.w.b_mop;
    const elem_t* src = val ? hv2 : ha2;
    const RowA<kHid> RH(r, h);
    f32x16 acc = acc_init(bias, blk * 32, h);
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) acc = mfma(W[(blk * 8 + ks) * 64 + lane], rowf(src, RH, 0, ks), acc);
    if constexpr (!kBiasFirst) acc += bias_init(bias, blk * 32, h);
    float* dst = (val ? vl : ml) + r * kAP + blk * 32;
#pragma unroll
    for (int g = 0; g < 16; g += 4) {   // positions 16 s + 8 h + i hold atoms feat(0, g, h) (natural order)
      const int m = (g & 3) + 8 * (g >> 2) + 4 * h;
      *reinterpret_cast<f32x4*>(dst + m) = f32x4{acc[g], acc[g + 1], acc[g + 2], acc[g + 3]};
    }
  }
  __syncthreads();

  // ---------------- the wave's actions: logits, softmax over atoms, expected value; argmax
  {
    const frag8* AO = reinterpret_cast<const frag8*>(a.w.ao);
    const RowA<kHid> RH(r, h);
    frag8 bh[kHid / 16];
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) bh[ks] = rowf(ha2, RH, 0, ks);
    // base = v - mean, and the support, for this lane's atoms: block b, register g
    float base[2][16], zz[2][16];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 16; g += 4) {
        const int m = b * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        const f32x4 vv = *reinterpret_cast<const f32x4*>(vl + r * kAP + m);
        const f32x4 mm = *reinterpret_cast<const f32x4*>(ml + r * kAP + m);
        const f32x4 z4 = *reinterpret_cast<const f32x4*>(L.z + m);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          base[b][g + i] = vv[i] - mm[i];
          zz[b][g + i] = z4[i];
        }
      }
    int pick = -1;
    if constexpr (MODE == RB_PICK) pick = static_cast<int>(io.act_idx[rr]);
    float bq = -INFINITY;
    int bk = 1 << 20;
    for (int k = w; k < kActs; k += kNW) {
      f32x16 acc[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[b] = acc_init(a.w.b_aop + k * kAP, b * 32, h);
#pragma unroll
        for (int ks = 0; ks < kHid / 16; ++ks) acc[b] = mfma(AO[((k * 2 + b) * 8 + ks) * 64 + lane], bh[ks], acc[b]);
        if constexpr (!kBiasFirst) acc[b] += bias_init(a.w.b_aop + k * kAP, b * 32, h);
      }
      float q[2][16], mx = -INFINITY;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int m = b * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
          q[b][g] = m < kAtoms ? acc[b][g] + base[b][g] : -INFINITY;
          mx = fmaxf(mx, q[b][g]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f, sz = 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
#if ASVRL_OPERAND_F32
          const float e = expf(q[b][g] - mx);
#else
          const float e = __expf(q[b][g] - mx);
#endif
          q[b][g] = e;
          se += e;
          sz += e * zz[b][g];
        }
      se = half_sum(se);
      sz = half_sum(sz);
      const float Q = sz / se;
      if (Q > bq) {   // actions ascend within the wave: ties keep the first
        bq = Q;
        bk = k;
      }
      if constexpr (MODE == RB_PICK) {
        if (k == pick && valid) {
          float* po = io.p_out + rr * kAtoms;
          const float inv = 1.f / se;
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
              const int m = b * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
              if (m < kAtoms) po[m] = q[b][g] * inv;
            }
        }
      }
    }
    if constexpr (MODE != RB_PICK) {
      if (h == 0) {
        L.best_q[w][r] = bq;
        L.best_k[w][r] = bk;
      }
    }
  }
  if constexpr (MODE == RB_PICK) return;
  __syncthreads();
  if (threadIdx.x >= 32 || !valid) return;
  float bq = L.best_q[0][r];
  int bk = L.best_k[0][r];
#pragma unroll
  for (int v = 1; v < kNW; ++v) {
    const float q = L.best_q[v][r];
    const int k = L.best_k[v][r];
    if (q > bq || (q == bq && k < bk)) {
      bq = q;
      bk = k;
    }
  }
  if constexpr (MODE == RB_ARGMAX) {
    io.act_idx[row] = bk;
  } else {
    // epsilon-greedy (agent.py:318-322): greedy iff random() > eps, else a uniform action; eps: the
    // linear schedule of the device step counter (trainer.py:257-264); the draws of rainbow_act_kernel
    double act = static_cast<double>(bk);
    if (io.step_dev != nullptr) {
      const uint64_t step = static_cast<uint64_t>(*io.step_dev);
      const double progress = static_cast<double>(step) * io.eps_steps_per_count / io.eps_total;
      const double eps = progress < io.eps_fraction
                             ? io.eps_initial + (progress / io.eps_fraction) * (io.eps_final - io.eps_initial)
                             : io.eps_final;
      const U4 u = philox4x32_10(U4{static_cast<uint32_t>(row), static_cast<uint32_t>(step),
                                    static_cast<uint32_t>(step >> 32), 0x5A1Bu},
                                 static_cast<uint32_t>(io.seed), static_cast<uint32_t>(io.seed >> 32));
      const double c = (static_cast<double>(u.x >> 8) + 1.0) * (1.0 / 16777216.0);   // (0, 1]
      if (!(c > eps)) act = static_cast<double>(u.y % kActs);
    }
    io.act_out[static_cast<int64_t>(row) * io.ld_act] = act;
    if (io.act_idx != nullptr) io.act_idx[row] = bk;
  }
}

// ------------------------------------------------------------------ packing
// Fragment images (asvrl_mfma.h frag_rc) of the encoders (256 x 32, input-fed) and the six composed
// NoisyLinear layers (chained): value / advantage hidden layers, the value output (51 rows, zero to 64),
// the action-mean of the advantage output (row i = mean_k Wao[51 k + i]), and the advantage output with
// each action's 51 rows zero-padded to 64; biases to the padded layouts, position order for the hidden
// layers' accumulator initialisation (bias_init reads position order).
constexpr int kImgEnc = kEnc * kObsK, kImgH1 = kHid * kEnc, kImgH2 = kHid * kHid, kImgO = kAP * kHid,
              kImgAO = kActs * kAP * kHid;
constexpr int kPackImg = kImgEnc + 2 * kImgH1 + 2 * kImgH2 + 2 * kImgO + kImgAO;
constexpr int kPackBias = kEnc + 4 * kHid + 2 * kAP + kActs * kAP;

__device__ float enc_w(const AsvRainbowSrc& s, int m, int k) {
  if (m < kSelfF) return k < kSelfIn ? s.self_w[m * kSelfIn + k] : 0.f;
  const int o = obj_of(m), j = (m - kSelfF) % kObjF, c = k - kSelfIn - kObjIn * o;
  return (c >= 0 && c < kObjIn) ? s.obj_w[j * kObjIn + c] : 0.f;
}

__device__ float out_row(const float* W, int rows, int row, int col) {
  return row < rows ? W[row * kHid + col] : 0.f;
}

__global__ __launch_bounds__(256) void rainbow_pack_kernel(AsvRainbowSrc s, AsvRainbowImgOut o) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < kPackImg) {
    int e = t, row, col;
    elem_t* dst;
    float v;
    if (e < kImgEnc) {
      frag_rc(e, kObsK, false, row, col);
      v = enc_w(s, row, col);
      dst = bp(o.enc) + e;
    } else if ((e -= kImgEnc) < 2 * kImgH1) {
      const int which = e / kImgH1, f = e % kImgH1;
      frag_rc(f, kEnc, true, row, col);
      v = (which ? s.w_a1 : s.w_v1)[row * kEnc + col];
      dst = bp(which ? o.a1 : o.v1) + f;
    } else if ((e -= 2 * kImgH1) < 2 * kImgH2) {
      const int which = e / kImgH2, f = e % kImgH2;
      frag_rc(f, kHid, true, row, col);
      v = (which ? s.w_a2 : s.w_v2)[row * kHid + col];
      dst = bp(which ? o.a2 : o.v2) + f;
    } else if ((e -= 2 * kImgH2) < kImgO) {
      frag_rc(e, kHid, true, row, col);
      v = out_row(s.w_vo, kAtoms, row, col);
      dst = bp(o.vo) + e;
    } else if ((e -= kImgO) < kImgO) {
      frag_rc(e, kHid, true, row, col);
      float acc = 0.f;
      if (row < kAtoms)
        for (int k = 0; k < kActs; ++k) acc += s.w_ao[(k * kAtoms + row) * kHid + col];
      v = acc / static_cast<float>(kActs);
      dst = bp(o.mo) + e;
    } else {
      e -= kImgO;
      frag_rc(e, kHid, true, row, col);   // row = 64 k + atom
      const int k = row / kAP, m = row % kAP;
      v = m < kAtoms ? s.w_ao[(k * kAtoms + m) * kHid + col] : 0.f;
      dst = bp(o.ao) + e;
    }
    *dst = (elem_t)v;
    return;
  }
  int b = t - kPackImg;
  if (b >= kPackBias) return;
  if (b < kEnc) {
    const int m = b;
    o.b_enc[m] = m < kSelfF ? s.self_b[m] : s.obj_b[(m - kSelfF) % kObjF];
  } else if ((b -= kEnc) < 4 * kHid) {
    const int which = b / kHid, i = b % kHid;
    const float* src = which == 0 ? s.b_v1 : which == 1 ? s.b_a1 : which == 2 ? s.b_v2 : s.b_a2;
    float* dst = which == 0 ? o.b_v1p : which == 1 ? o.b_a1p : which == 2 ? o.b_v2p : o.b_a2p;
    dst[swap23(i)] = src[i];
  } else if ((b -= 4 * kHid) < kAP) {
    o.b_vop[swap23(b)] = b < kAtoms ? s.b_vo[b] : 0.f;
  } else if ((b -= kAP) < kAP) {
    float acc = 0.f;
    if (b < kAtoms)
      for (int k = 0; k < kActs; ++k) acc += s.b_ao[k * kAtoms + b];
    o.b_mop[swap23(b)] = acc / static_cast<float>(kActs);
  } else {
    b -= kAP;
    const int k = b / kAP, m = b % kAP;
    o.b_aop[k * kAP + swap23(m)] = m < kAtoms ? s.b_ao[k * kAtoms + m] : 0.f;
  }
}

int launch_net(int mode, const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  RbArgs a{*w, *io};
  const dim3 grid((io->N + 31) / 32), block(kNW * 64);
  hipStream_t st = as_stream(stream);
  if (mode == RB_ACT) hipLaunchKernelGGL(rainbow_net_kernel<RB_ACT>, grid, block, 0, st, a);
  else if (mode == RB_ARGMAX) hipLaunchKernelGGL(rainbow_net_kernel<RB_ARGMAX>, grid, block, 0, st, a);
  else hipLaunchKernelGGL(rainbow_net_kernel<RB_PICK>, grid, block, 0, st, a);
  return check_launch("asvrl_rainbow_net");
}

int check_img(const AsvRainbowImg* w, const AsvRainbowNetIO* io) {
  ASVRL_REQUIRE(w && io, "asvrl_rainbow_net: null argument");
  ASVRL_REQUIRE(w->enc && w->b_enc && w->v1 && w->a1 && w->v2 && w->a2 && w->vo && w->mo && w->ao && w->b_v1p &&
                    w->b_a1p && w->b_v2p && w->b_a2p && w->b_vop && w->b_mop && w->b_aop,
                "asvrl_rainbow_net: null weight image");
  ASVRL_REQUIRE(io->x && io->ldx >= 40 && io->ldx % 4 == 0 && reinterpret_cast<uintptr_t>(io->x) % 16 == 0,
                "asvrl_rainbow_net: obs rows must be 16-byte aligned with ldx >= 40");
  ASVRL_REQUIRE(io->support, "asvrl_rainbow_net: null support");
  return 0;
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_rainbow_pack(const AsvRainbowSrc* src, const AsvRainbowImgOut* img, void* stream) {
  ASVRL_REQUIRE(src && img, "asvrl_rainbow_pack: null argument");
  ASVRL_REQUIRE(src->self_w && src->self_b && src->obj_w && src->obj_b && src->w_v1 && src->b_v1 && src->w_a1 &&
                    src->b_a1 && src->w_v2 && src->b_v2 && src->w_a2 && src->b_a2 && src->w_vo && src->b_vo &&
                    src->w_ao && src->b_ao,
                "asvrl_rainbow_pack: null source weight");
  ASVRL_REQUIRE(img->enc && img->b_enc && img->v1 && img->a1 && img->v2 && img->a2 && img->vo && img->mo && img->ao &&
                    img->b_v1p && img->b_a1p && img->b_v2p && img->b_a2p && img->b_vop && img->b_mop && img->b_aop,
                "asvrl_rainbow_pack: null image");
  const int total = kPackImg + kPackBias;
  hipLaunchKernelGGL(rainbow_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), *src, *img);
  return check_launch("asvrl_rainbow_pack");
}

extern "C" int asvrl_rainbow_net_act(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  if (int rc = check_img(w, io)) return rc;
  ASVRL_REQUIRE(io->act_out && io->ld_act >= 1, "asvrl_rainbow_net_act: needs act_out");
  ASVRL_REQUIRE(io->step_dev == nullptr || (io->eps_total > 0.0 && io->eps_fraction > 0.0),
                "asvrl_rainbow_net_act: bad epsilon schedule");
  if (io->N <= 0) return 0;
  return launch_net(RB_ACT, w, io, stream);
}

extern "C" int asvrl_rainbow_net_argmax(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  if (int rc = check_img(w, io)) return rc;
  ASVRL_REQUIRE(io->act_idx, "asvrl_rainbow_net_argmax: needs act_idx");
  if (io->N <= 0) return 0;
  return launch_net(RB_ARGMAX, w, io, stream);
}

extern "C" int asvrl_rainbow_net_pick(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  if (int rc = check_img(w, io)) return rc;
  ASVRL_REQUIRE(io->act_idx && io->p_out, "asvrl_rainbow_net_pick: needs act_idx and p_out");
  if (io->N <= 0) return 0;
  return launch_net(RB_PICK, w, io, stream);
}
