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

// The training pass keeps every activation image until its mask has been taken (the masks then live
// in registers): f, later dz2 | h1, later dz1 | h2 | v, mean logits, later the dq image + dq (f32).
struct RbTrainLds {
  elem_t x0[32 * kEnc];
  elem_t h1[2][32 * kHid];
  elem_t h2[2][32 * kHid];
  float vm[2][32 * kAP];
  float z[kAP];
  int act[32];
};
static_assert(2 * 32 * kAP * sizeof(float) >= 32 * kAP * (sizeof(elem_t) + sizeof(float)), "dq images fit over vm");

// object index of encoder feature m (>= 56)
__device__ __forceinline__ int obj_of(int m) { return (m - kSelfF) / kObjF; }

// object ob's mask factor (ob wave-uniform; -1, the self encoder, and kObjN give 1): selects on a scalar
// condition, no lane-divergent branches
static_assert(kSelfF >= 32 && kObjF >= 32, "a 32-feature block spans at most two encoders");
__device__ __forceinline__ float obj_sel(int ob, const float (&mf)[kObjN]) {
  float f = 1.f;
#pragma unroll
  for (int o = 0; o < kObjN; ++o) f = ob == o ? mf[o] : f;
  return f;
}

// natural atom index of register g of block b in lane half h
__device__ __forceinline__ int atom_of(int b, int g, int h) { return b * 32 + (g & 3) + 8 * (g >> 2) + 4 * h; }

// ---------------- forward phases (wave w of 4), shared by the inference and training kernels. SAVE:
// also the activations to HBM (store16: all 64 lanes call it; dst nullptr for rows past N) and the
// lane's ReLU masks (bit 8 s + i of a block = register 8 s + i positive).

// encoders -> f (wave w: blocks 2w, 2w + 1) into x0
template <bool SAVE>
__device__ __forceinline__ void phase_encode(const AsvRainbowImg& W, const float* xr, elem_t* x0, int w, int lane,
                                             elem_t* f_row, uint32_t& fmask) {
  const int h = lane >> 5, r = lane & 31;
  frag8 bx[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(xr + ks * 16 + 8 * h);
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + ks * 16 + 8 * h + 4);
    const float e[8] = {u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
    bx[ks] = pack8(e);
  }
  float mf[kObjN];   // masked_fill(mask < 0.5, 0) as a factor per object
#pragma unroll
  for (int o = 0; o < kObjN; ++o) mf[o] = xr[32 + o] < 0.5f ? 0.f : 1.f;
  const frag8* ENC = reinterpret_cast<const frag8*>(W.enc);
  const RowA<kEnc> RA(r, h);
  fmask = 0;
  w = __builtin_amdgcn_readfirstlane(w);   // wave-uniform: the block / object indices below are scalar work
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int mb = 2 * w + q;
    f32x16 acc = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) acc = mfma(ENC[(mb * 2 + ks) * 64 + lane], bx[ks], acc);
    // the block spans at most two encoders: A (from its first feature) up to the next boundary, then
    // A + 1; the lane's feature 8k + i + 4h of the block is in A iff 8k + i < lim (one select per element)
    const int m_lo = mb * 32;
    const int obA = m_lo < kSelfF ? -1 : obj_of(m_lo);
    const int lim = kSelfF + kObjF * (obA + 1) - m_lo - 4 * h;
    const float fA = obj_sel(obA, mf), fB = obj_sel(obA + 1, mf);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int g = 8 * s + i;
        const int m = feat(mb, g, h);
        const float keep = (g & 3) + 8 * (g >> 2) < lim ? fA : fB;
        v[i] = relu(acc[8 * s + i] + W.b_enc[m]) * keep;
        if (SAVE && v[i] > 0.f) fmask |= 1u << (16 * q + 8 * s + i);
      }
      rows(x0, RA, 0, 2 * mb + s, pack8(v));
      if constexpr (SAVE) store16(f_row != nullptr ? f_row + mb * 32 + 16 * s : nullptr, v, h);
    }
  }
}

// MFMA chains whose A operands (weight fragment images) come from L2: t < T steps, step t's fragment(s)
// fetched D steps ahead into a ring, one scheduling fence per step -- otherwise every MFMA waits for its
// own global load (ASVRL_RB_READ_AHEAD = D; same MFMA order, bit-identical). D = 4 (default): Rainbow step
// 0.489-0.494 -> 0.411-0.413 ms at 8192 envs (profiles/r02_rb_read_ahead_ab.txt); D = 8 no better.
#ifndef ASVRL_RB_READ_AHEAD
#define ASVRL_RB_READ_AHEAD 4
#endif
template <int T, int NA, class AF, class MF>
__device__ __forceinline__ void mfma_ring(AF af, MF mf) {
  constexpr int D = ASVRL_RB_READ_AHEAD < T ? ASVRL_RB_READ_AHEAD : T;
  if constexpr (D == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      frag8 A[NA];
      af(t, A);
      mf(t, A);
    }
  } else {
    frag8 q[D][NA];
#pragma unroll
    for (int t = 0; t < D; ++t) af(t, q[t]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      mf(t, q[t % D]);
      if (t + D < T) af(t + D, q[t % D]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// one hidden layer pair (value, advantage streams; wave w: block w of each): out = relu(W in + b)
template <int K, bool SAVE>
__device__ __forceinline__ void phase_hidden(const void* wv, const void* wa, const float* bv, const float* ba,
                                             const elem_t* inv, const elem_t* ina, elem_t* outv, elem_t* outa, int w,
                                             int lane, elem_t* sv_row, elem_t* sa_row, uint32_t& mask) {
  const int h = lane >> 5, r = lane & 31;
  const frag8* V = reinterpret_cast<const frag8*>(wv);
  const frag8* A = reinterpret_cast<const frag8*>(wa);
  const RowA<K> RX(r, h);
  const RowA<kHid> RH(r, h);
  f32x16 av = acc_init(bv, w * 32, h), aa = acc_init(ba, w * 32, h);
  mfma_ring<K / 16, 2>(
      [&](int ks, frag8(&q)[2]) {
        q[0] = V[(w * (K / 16) + ks) * 64 + lane];
        q[1] = A[(w * (K / 16) + ks) * 64 + lane];
      },
      [&](int ks, const frag8(&q)[2]) {
        const frag8 b0 = rowf(inv, RX, 0, ks);
        av = mfma(q[0], b0, av);
        const frag8 b1 = inv == ina ? b0 : rowf(ina, RX, 0, ks);
        aa = mfma(q[1], b1, aa);
      });
  if constexpr (!kBiasFirst) {
    av += bias_init(bv, w * 32, h);
    aa += bias_init(ba, w * 32, h);
  }
  mask = 0;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float fv[8], fa[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fv[i] = relu(av[8 * s + i]);
      fa[i] = relu(aa[8 * s + i]);
      if (SAVE) mask |= (fv[i] > 0.f ? 1u : 0u) << (8 * s + i) | (fa[i] > 0.f ? 1u : 0u) << (16 + 8 * s + i);
    }
    rows(outv, RH, 0, 2 * w + s, pack8(fv));
    rows(outa, RH, 0, 2 * w + s, pack8(fa));
    if constexpr (SAVE) {
      store16(sv_row != nullptr ? sv_row + w * 32 + 16 * s : nullptr, fv, h);
      store16(sa_row != nullptr ? sa_row + w * 32 + 16 * s : nullptr, fa, h);
    }
  }
}

// v (waves 0, 1: atom blocks 0, 1) and the action-mean logits (waves 2, 3) -> f32 [32][64], natural order
__device__ __forceinline__ void phase_vm(const AsvRainbowImg& W, const elem_t* hv2, const elem_t* ha2, float* vl,
                                         float* ml, int w, int lane) {
  const int h = lane >> 5, r = lane & 31;
  const bool val = w < 2;
  const int blk = w & 1;
  const frag8* M = reinterpret_cast<const frag8*>(val ? W.vo : W.mo);
  const float* bias = val ? W.b_vop : W.b_mop;
  const elem_t* src = val ? hv2 : ha2;
  const RowA<kHid> RH(r, h);
  f32x16 acc = acc_init(bias, blk * 32, h);
  mfma_ring<kHid / 16, 1>([&](int ks, frag8(&q)[1]) { q[0] = M[(blk * 8 + ks) * 64 + lane]; },
                          [&](int ks, const frag8(&q)[1]) { acc = mfma(q[0], rowf(src, RH, 0, ks), acc); });
  if constexpr (!kBiasFirst) acc += bias_init(bias, blk * 32, h);
  float* dst = (val ? vl : ml) + r * kAP + blk * 32;
#pragma unroll
  for (int g = 0; g < 16; g += 4) {   // registers g .. g + 3 hold atoms atom_of(0, g, h) .. + 3
    const int m = atom_of(0, g, h);
    *reinterpret_cast<f32x4*>(dst + m) = f32x4{acc[g], acc[g + 1], acc[g + 2], acc[g + 3]};
  }
}

// base = v - mean and the support for this lane's atoms (block b, register g)
__device__ __forceinline__ void load_base(const float* vl, const float* ml, const float* z, int r, int h,
                                          float (&base)[2][16], float (&zz)[2][16]) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int g = 0; g < 16; g += 4) {
      const int m = atom_of(b, g, h);
      const f32x4 vv = *reinterpret_cast<const f32x4*>(vl + r * kAP + m);
      const f32x4 mm = *reinterpret_cast<const f32x4*>(ml + r * kAP + m);
      const f32x4 z4 = *reinterpret_cast<const f32x4*>(z + m);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        base[b][g + i] = vv[i] - mm[i];
        zz[b][g + i] = z4[i];
      }
    }
}

// action k's 51 advantage logits (two 32-atom blocks) from the ha2 fragments
__device__ __forceinline__ void action_logits(const AsvRainbowImg& W, const frag8 (&bh)[kHid / 16], int k, int lane,
                                              f32x16 (&acc)[2]) {
  const int h = lane >> 5;
  const frag8* AO = reinterpret_cast<const frag8*>(W.ao);
#pragma unroll
  for (int b = 0; b < 2; ++b) acc[b] = acc_init(W.b_aop + k * kAP, b * 32, h);
  mfma_ring<2 * (kHid / 16), 1>(
      [&](int t, frag8(&q)[1]) { q[0] = AO[((k * 2 + t / 8) * 8 + t % 8) * 64 + lane]; },
      [&](int t, const frag8(&q)[1]) { acc[t / 8] = mfma(q[0], bh[t % 8], acc[t / 8]); });
#pragma unroll
  for (int b = 0; b < 2; ++b)
    if constexpr (!kBiasFirst) acc[b] += bias_init(W.b_aop + k * kAP, b * 32, h);
}

__device__ __forceinline__ float fexp(float x) {
#if ASVRL_OPERAND_F32
  return expf(x);
#else
  return __expf(x);
#endif
}

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
  uint32_t unused = 0;
  phase_encode<false>(a.w, io.x + rr * io.ldx, L.x0, w, lane, nullptr, unused);
  __syncthreads();
  phase_hidden<kEnc, false>(a.w.v1, a.w.a1, a.w.b_v1p, a.w.b_a1p, L.x0, L.x0, L.h1[0], L.h1[1], w, lane, nullptr,
                            nullptr, unused);
  __syncthreads();
  elem_t* const hv2 = L.x0;               // x0 is dead after the first hidden layers
  elem_t* const ha2 = L.x0 + 32 * kHid;
  phase_hidden<kHid, false>(a.w.v2, a.w.a2, a.w.b_v2p, a.w.b_a2p, L.h1[0], L.h1[1], hv2, ha2, w, lane, nullptr,
                            nullptr, unused);
  __syncthreads();
  float* const vl = reinterpret_cast<float*>(&L.h1[0][0]);   // h1: last read by layer 2, behind the barrier
  float* const ml = vl + 32 * kAP;
  phase_vm(a.w, hv2, ha2, vl, ml, w, lane);
  __syncthreads();

  // ---------------- the wave's actions: logits, softmax over atoms, expected value; argmax
  {
    const RowA<kHid> RH(r, h);
    frag8 bh[kHid / 16];
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) bh[ks] = rowf(ha2, RH, 0, ks);
    float base[2][16], zz[2][16];
    load_base(vl, ml, L.z, r, h, base, zz);
    int pick = -1;
    if constexpr (MODE == RB_PICK) pick = static_cast<int>(io.act_idx[rr]);
    float bq = -INFINITY;
    int bk = 1 << 20;
    for (int k = w; k < kActs; k += kNW) {
      f32x16 acc[2];
      action_logits(a.w, bh, k, lane, acc);
      float q[2][16], mx = -INFINITY;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          q[b][g] = atom_of(b, g, h) < kAtoms ? acc[b][g] + base[b][g] : -INFINITY;
          mx = fmaxf(mx, q[b][g]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f, sz = 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float e = fexp(q[b][g] - mx);
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
            for (int g = 0; g < 16; ++g)
              if (atom_of(b, g, h) < kAtoms) po[atom_of(b, g, h)] = q[b][g] * inv;
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

// ---------------- train_Rainbow's training pass (agent.py:613-636) on the online net, rows = s.
// Forward as above saving the weight-gradient inputs; the wave owning action a_b computes row b's
// loss_b = -sum m log p (p = softmax(q[a_b])) and dq = grad_scale w_b (p sum(m) - m) (the gradient of
// grad_scale sum_b w_b loss_b with respect to q[a_b]); q = v + a - mean_k a gives dv = dq and
// da[k] = dq (1{k = a_b} - 1/25), so
//   dh2v = Wvo^T dq,   dh2a = Wao[a_b]^T dq - mean_k(Wao[k])^T dq
// (the first term as 25 MFMA passes over the action-masked dq image), then relu masks, W2^T, W1^T down
// to the encoders' pre-activations.
template <int K>
__device__ __forceinline__ void phase_back(const void* wvt, const void* wat, const elem_t* dinv, const elem_t* dina,
                                           int mb, int lane, f32x16& dv, f32x16& da) {
  const int h = lane >> 5, r = lane & 31;
  const frag8* VT = reinterpret_cast<const frag8*>(wvt);
  const frag8* AT = reinterpret_cast<const frag8*>(wat);
  const RowA<K> RD(r, h);
  dv = f32x16{};
  da = f32x16{};
  mfma_ring<K / 16, 2>(
      [&](int ks, frag8(&q)[2]) {
        q[0] = VT[(mb * (K / 16) + ks) * 64 + lane];
        q[1] = AT[(mb * (K / 16) + ks) * 64 + lane];
      },
      [&](int ks, const frag8(&q)[2]) {
        dv = mfma(q[0], rowf(dinv, RD, 0, ks), dv);
        da = mfma(q[1], rowf(dina, RD, 0, ks), da);
      });
}

__global__ __launch_bounds__(kNW * 64) void rainbow_train_kernel(RbArgs a) {
  __shared__ __attribute__((aligned(16))) RbTrainLds L;
  const AsvRainbowNetIO& io = a.io;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int row0 = blockIdx.x * 32;
  const int row = row0 + r;
  const bool valid = row < io.N;
  const int64_t rr = valid ? row : io.N - 1;
  if (threadIdx.x < kAP) L.z[threadIdx.x] = threadIdx.x < kAtoms ? io.support[threadIdx.x] : 0.f;
  if (threadIdx.x < 32) {
    const int k = static_cast<int>(io.actions[(row0 + threadIdx.x < io.N ? row0 + threadIdx.x : io.N - 1) * io.ld_rd]);
    L.act[threadIdx.x] = k < 0 ? 0 : (k >= kActs ? kActs - 1 : k);
  }
  auto orow = [&](void* base, int width) -> elem_t* {
    return valid ? bp(base) + static_cast<int64_t>(row) * width : nullptr;
  };
  // ---------------- forward, saving f, hv1, ha1, hv2, ha2 (and xb) with the ReLU masks in registers
  const float* xr = io.x + rr * io.ldx;
  if (w == 0 && valid) {   // xb: obs columns 0 .. 31 in the operand type (the encoder fold's input)
    elem_t* xo = bp(io.xb) + static_cast<int64_t>(row) * kObsK + 16 * h;
#pragma unroll
    for (int j = 0; j < 16; ++j) xo[j] = (elem_t)xr[16 * h + j];
  }
  uint32_t fmask, m1, m2;
  phase_encode<true>(a.w, xr, L.x0, w, lane, orow(io.f, kEnc), fmask);
  __syncthreads();
  phase_hidden<kEnc, true>(a.w.v1, a.w.a1, a.w.b_v1p, a.w.b_a1p, L.x0, L.x0, L.h1[0], L.h1[1], w, lane,
                           orow(io.hv1, kHid), orow(io.ha1, kHid), m1);
  __syncthreads();
  phase_hidden<kHid, true>(a.w.v2, a.w.a2, a.w.b_v2p, a.w.b_a2p, L.h1[0], L.h1[1], L.h2[0], L.h2[1], w, lane,
                           orow(io.hv2, kHid), orow(io.ha2, kHid), m2);
  __syncthreads();
  float* const vl = L.vm[0];
  float* const ml = L.vm[1];
  phase_vm(a.w, L.h2[0], L.h2[1], vl, ml, w, lane);
  __syncthreads();

  // ---------------- loss and dq of each row, by the wave owning its action
  const int act_r = L.act[r];
  {
    const RowA<kHid> RH(r, h);
    frag8 bh[kHid / 16];
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) bh[ks] = rowf(L.h2[1], RH, 0, ks);
    float base[2][16], zz[2][16];
    load_base(vl, ml, L.z, r, h, base, zz);
    float mv[2][16], wgt = 0.f;
    {
      const float* mr = io.m + rr * kAtoms;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) mv[b][g] = atom_of(b, g, h) < kAtoms ? mr[atom_of(b, g, h)] : 0.f;
      wgt = io.weights[rr * io.ld_rd];
    }
    float sm = 0.f;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 16; ++g) sm += mv[b][g];
    sm = half_sum(sm);
    __syncthreads();   // every wave holds its base: vm becomes the dq images
    elem_t* const dqi = reinterpret_cast<elem_t*>(L.vm[0]);   // [32][64] chained position order
    float* const dqf = L.vm[1];                                // [32][64] natural order
    const RowA<kAP> RQ(r, h);
    for (int k = w; k < kActs; k += kNW) {
      f32x16 acc[2];
      action_logits(a.w, bh, k, lane, acc);
      if (act_r != k) continue;   // lane-divergent from here: no cross-lane ops other than within the row pair
      float q[2][16], mx = -INFINITY;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          q[b][g] = atom_of(b, g, h) < kAtoms ? acc[b][g] + base[b][g] : -INFINITY;
          mx = fmaxf(mx, q[b][g]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g) se += fexp(q[b][g] - mx);
      se = half_sum(se);
      const float lse = mx + logf(se);
      float l = 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 16; ++g)
          if (atom_of(b, g, h) < kAtoms) l -= mv[b][g] * (q[b][g] - lse);
      l = half_sum(l);
      if (valid && h == 0) io.loss[row] = l;
      const float sc = valid ? wgt * io.grad_scale : 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int g = 8 * s + i;
            const bool on = atom_of(b, g, h) < kAtoms;
            const float d = on ? (fexp(q[b][g] - lse) * sm - mv[b][g]) * sc : 0.f;
            o[i] = d;
            dqf[r * kAP + atom_of(b, g, h)] = d;
          }
          rows(dqi, RQ, 0, 2 * b + s, pack8(o));
        }
    }
  }
  __syncthreads();
  const elem_t* const dqi = reinterpret_cast<const elem_t*>(L.vm[0]);
  const float* const dqf = L.vm[1];

  // ---------------- dZ of the output layers to HBM: dzv [N][64] = dq, dza [N][1280] = da (51 per action)
  for (int c = threadIdx.x; c < 32 * (kAP / 8); c += kNW * 64) {
    const int rw = c / (kAP / 8), ch = c % (kAP / 8);
    if (row0 + rw >= io.N) continue;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = dqf[rw * kAP + 8 * ch + i];
    *reinterpret_cast<frag8*>(bp(io.dzv) + static_cast<int64_t>(row0 + rw) * kAP + 8 * ch) = pack8(o);
  }
  constexpr int kDa = 1280;
  for (int c = threadIdx.x; c < 32 * (kDa / 8); c += kNW * 64) {
    const int rw = c / (kDa / 8), ch = c % (kDa / 8);
    if (row0 + rw >= io.N) continue;
    const int ar = L.act[rw];
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int col = 8 * ch + i, k = col / kAtoms, m = col - k * kAtoms;
      const float d = col < kActs * kAtoms ? dqf[rw * kAP + m] : 0.f;
      o[i] = col < kActs * kAtoms ? (k == ar ? d - d / static_cast<float>(kActs) : -d / static_cast<float>(kActs)) : 0.f;
    }
    *reinterpret_cast<frag8*>(bp(io.dza) + static_cast<int64_t>(row0 + rw) * kDa + 8 * ch) = pack8(o);
  }

  // ---------------- dh2 (wave w: block w) -> dz2 into x0's space (f is only needed as the mask now)
  elem_t* const dz2v = L.x0;
  elem_t* const dz2a = L.x0 + 32 * kHid;
  {
    const RowA<kAP> RQ(r, h);
    const RowA<kHid> RH(r, h);
    const frag8* VOT = reinterpret_cast<const frag8*>(a.w.vot);
    const frag8* MOT = reinterpret_cast<const frag8*>(a.w.mot);
    const frag8* AOT = reinterpret_cast<const frag8*>(a.w.aot);
    frag8 bq[kAP / 16];
#pragma unroll
    for (int ks = 0; ks < kAP / 16; ++ks) bq[ks] = rowf(dqi, RQ, 0, ks);
    f32x16 dv = f32x16{}, da = f32x16{};
    mfma_ring<kAP / 16, 2>(
        [&](int ks, frag8(&q)[2]) {
          q[0] = VOT[(w * 4 + ks) * 64 + lane];
          q[1] = MOT[(w * 4 + ks) * 64 + lane];
        },
        [&](int ks, const frag8(&q)[2]) {
          dv = mfma(q[0], bq[ks], dv);
          da = mfma(q[1], bq[ks], da);   // - mean_k Wao[k]^T dq
        });
    for (int k = 0; k < kActs; ++k) {
      if (__builtin_amdgcn_readfirstlane(__ballot(act_r == k) != 0) == 0) continue;   // action absent from the tile
      const frag8 zero{};
      mfma_ring<kAP / 16, 1>([&](int ks, frag8(&q)[1]) { q[0] = AOT[((k * 4 + w) * 4 + ks) * 64 + lane]; },
                             [&](int ks, const frag8(&q)[1]) { da = mfma(q[0], act_r == k ? bq[ks] : zero, da); });
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float fv[8], fa[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        fv[i] = (m2 >> (8 * s + i)) & 1u ? dv[8 * s + i] : 0.f;
        fa[i] = (m2 >> (16 + 8 * s + i)) & 1u ? da[8 * s + i] : 0.f;
      }
      rows(dz2v, RH, 0, 2 * w + s, pack8(fv));
      rows(dz2a, RH, 0, 2 * w + s, pack8(fa));
      elem_t* sv = orow(io.dz2v, kHid);
      elem_t* sa = orow(io.dz2a, kHid);
      store16(sv != nullptr ? sv + w * 32 + 16 * s : nullptr, fv, h);
      store16(sa != nullptr ? sa + w * 32 + 16 * s : nullptr, fa, h);
    }
  }
  __syncthreads();

  // ---------------- dh1 = W2^T dz2 (block w) -> dz1 into h1's space
  elem_t* const dz1v = L.h1[0];
  elem_t* const dz1a = L.h1[1];
  {
    f32x16 dv, da;
    phase_back<kHid>(a.w.v2t, a.w.a2t, dz2v, dz2a, w, lane, dv, da);
    const RowA<kHid> RH(r, h);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float fv[8], fa[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        fv[i] = (m1 >> (8 * s + i)) & 1u ? dv[8 * s + i] : 0.f;
        fa[i] = (m1 >> (16 + 8 * s + i)) & 1u ? da[8 * s + i] : 0.f;
      }
      rows(dz1v, RH, 0, 2 * w + s, pack8(fv));
      rows(dz1a, RH, 0, 2 * w + s, pack8(fa));
      elem_t* sv = orow(io.dz1v, kHid);
      elem_t* sa = orow(io.dz1a, kHid);
      store16(sv != nullptr ? sv + w * 32 + 16 * s : nullptr, fv, h);
      store16(sa != nullptr ? sa + w * 32 + 16 * s : nullptr, fa, h);
    }
  }
  __syncthreads();

  // ---------------- df = Wv1^T dz1v + Wa1^T dz1a (blocks 2w, 2w + 1) -> dz of the encoders
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    f32x16 dv, da;
    phase_back<kHid>(a.w.v1t, a.w.a1t, dz1v, dz1a, 2 * w + q, lane, dv, da);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float fv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fv[i] = (fmask >> (16 * q + 8 * s + i)) & 1u ? dv[8 * s + i] + da[8 * s + i] : 0.f;
      elem_t* sf = orow(io.dzf, kEnc);
      store16(sf != nullptr ? sf + (2 * w + q) * 32 + 16 * s : nullptr, fv, h);
    }
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
// the backward's transposed images (A = W^T, chained over the layer's outputs): vot, mot (-mean), aot,
// v2t, a2t, v1t, a1t
constexpr int kPackT = 2 * kImgO + kImgAO + 2 * kImgH2 + 2 * kImgH1;

__device__ float enc_w(const AsvRainbowSrc& s, int m, int k) {
  if (m < kSelfF) return k < kSelfIn ? s.self_w[m * kSelfIn + k] : 0.f;
  const int o = obj_of(m), j = (m - kSelfF) % kObjF, c = k - kSelfIn - kObjIn * o;
  return (c >= 0 && c < kObjIn) ? s.obj_w[j * kObjIn + c] : 0.f;
}

__device__ float out_row(const float* W, int rows, int row, int col) {
  return row < rows ? W[row * kHid + col] : 0.f;
}

__device__ void pack_transposed(const AsvRainbowSrc& s, const AsvRainbowImgOut& o, int e) {
  int row, col;
  float v;
  elem_t* dst;
  if (e < kImgO) {   // Wvo^T: M = 128 inputs, K = 64 atoms (51 + zeros)
    frag_rc(e, kAP, true, row, col);
    v = col < kAtoms ? s.w_vo[col * kHid + row] : 0.f;
    dst = bp(o.vot) + e;
  } else if ((e -= kImgO) < kImgO) {   // -mean_k Wao[k]^T
    frag_rc(e, kAP, true, row, col);
    float acc = 0.f;
    if (col < kAtoms)
      for (int k = 0; k < kActs; ++k) acc += s.w_ao[(k * kAtoms + col) * kHid + row];
    v = -(acc / static_cast<float>(kActs));
    dst = bp(o.mot) + e;
  } else if ((e -= kImgO) < kImgAO) {   // Wao[k]^T per action
    const int k = e / kImgO, f = e % kImgO;
    frag_rc(f, kAP, true, row, col);
    v = col < kAtoms ? s.w_ao[(k * kAtoms + col) * kHid + row] : 0.f;
    dst = bp(o.aot) + e;
  } else if ((e -= kImgAO) < 2 * kImgH2) {   // W2^T
    const int which = e / kImgH2, f = e % kImgH2;
    frag_rc(f, kHid, true, row, col);
    v = (which ? s.w_a2 : s.w_v2)[col * kHid + row];
    dst = bp(which ? o.a2t : o.v2t) + f;
  } else {   // W1^T: M = 256 inputs, K = 128 outputs
    e -= 2 * kImgH2;
    const int which = e / kImgH1, f = e % kImgH1;
    frag_rc(f, kHid, true, row, col);
    v = (which ? s.w_a1 : s.w_v1)[col * kEnc + row];
    dst = bp(which ? o.a1t : o.v1t) + f;
  }
  *dst = (elem_t)v;
}

__global__ __launch_bounds__(256) void rainbow_pack_kernel(AsvRainbowSrc s, AsvRainbowImgOut o) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= kPackImg + kPackBias) {
    if (t < kPackImg + kPackBias + kPackT && o.vot != nullptr) pack_transposed(s, o, t - kPackImg - kPackBias);
    return;
  }
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

int launch_train(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  RbArgs a{*w, *io};
  hipLaunchKernelGGL(rainbow_train_kernel, dim3((io->N + 31) / 32), dim3(kNW * 64), 0, as_stream(stream), a);
  return check_launch("asvrl_rainbow_net_train");
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
  const bool tr = img->vot != nullptr;
  ASVRL_REQUIRE(!tr || (img->mot && img->aot && img->v2t && img->a2t && img->v1t && img->a1t),
                "asvrl_rainbow_pack: the transposed images come all or none");
  const int total = kPackImg + kPackBias + (tr ? kPackT : 0);
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

extern "C" int asvrl_rainbow_net_train(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream) {
  if (int rc = check_img(w, io)) return rc;
  ASVRL_REQUIRE(w->vot && w->mot && w->aot && w->v2t && w->a2t && w->v1t && w->a1t,
                "asvrl_rainbow_net_train: needs the transposed images (asvrl_rainbow_pack with vot ... a1t)");
  ASVRL_REQUIRE(io->actions && io->weights && io->ld_rd >= 1 && io->m && io->loss,
                "asvrl_rainbow_net_train: needs actions, weights, m and loss");
  ASVRL_REQUIRE(io->xb && io->f && io->hv1 && io->ha1 && io->hv2 && io->ha2 && io->dzv && io->dza && io->dz2v &&
                    io->dz2a && io->dz1v && io->dz1a && io->dzf,
                "asvrl_rainbow_net_train: null activation / gradient image");
  if (io->N <= 0) return 0;
  return launch_train(w, io, stream);
}
