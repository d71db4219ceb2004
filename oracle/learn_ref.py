"""CPU restatement of rfarl's distributional learners (TEST INFRASTRUCTURE ONLY).

Functional torch-fp32 versions of the networks and update steps, written against weight
dicts keyed like the reference's state_dicts -- independent of the product's nn.Modules:
  ac_iqn_train   agent.py:386-432 (+ AC_IQN_model.py:284-323, 410-480)
  iqn_train      agent.py:434-476 (+ IQN_model.py:56-110)
  rainbow_train  agent.py:597-641 (+ Rainbow_model.py:17-139), C51 target m restated in
                 explicit per-atom loops (the reference's index_add_ order)
  adam_step      torch.optim.Adam defaults (single-tensor form), clip_grad_norm_
Pinned against tests/golden/learn_*.npz (captured from the reference). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline import this.
"""
import math

import numpy as np
import torch

F = torch.nn.functional


def _lin(w, p, x):
    return F.linear(x, w[p + ".weight"], w[p + ".bias"])


def _features(w, s_self, s_obj, s_mask, obj_feat=40, max_obj=5, obj_dim=5):
    B = s_self.shape[0]
    f1 = torch.relu(_lin(w, "self_encoder.0", s_self))
    f2 = torch.relu(_lin(w, "object_encoder.0", s_obj.reshape(B * max_obj, obj_dim))).view(B, max_obj, obj_feat)
    f2 = f2.masked_fill(s_mask.unsqueeze(-1) < 0.5, 0.0).reshape(B, max_obj * obj_feat)
    return torch.cat((f1, f2), 1)


def actor_forward(w, s):
    f = _features(w, *s)
    f = torch.relu(_lin(w, "hidden_layer", f))
    f = torch.relu(_lin(w, "hidden_layer_2", f))
    return torch.tensor(2.0 / torch.pi) * torch.atan(_lin(w, "output_layer", f))


def _cos(taus, n=64):
    pis = torch.FloatTensor([np.pi * i for i in range(n)]).view(1, 1, n)
    return torch.cos(taus * pis)


def critic_forward(w, s, a, taus):
    """taus (B, N, 1) -> quantiles (B, N)."""
    B, N = taus.shape[0], taus.shape[1]
    f = _features(w, *s)
    c = torch.relu(_lin(w, "cos_embedding", _cos(taus).view(B * N, 64))).view(B, N, -1)
    f = (f.unsqueeze(1) * c).view(B * N, -1)
    f = torch.relu(_lin(w, "hidden_layer", f))
    af = torch.relu(_lin(w, "action_encoder.0", a))
    f = (af.unsqueeze(1) * f.view(B, N, -1)).view(B * N, -1)
    f = torch.relu(_lin(w, "hidden_layer_2", f))
    return _lin(w, "output_layer", f).view(B, N)


def iqn_forward(w, s, taus, action_size=25):
    B, N = taus.shape[0], taus.shape[1]
    f = _features(w, *s)
    c = torch.relu(_lin(w, "cos_embedding", _cos(taus).view(B * N, 64))).view(B, N, -1)
    f = (f.unsqueeze(1) * c).view(B * N, -1)
    f = torch.relu(_lin(w, "hidden_layer", f))
    f = torch.relu(_lin(w, "hidden_layer_2", f))
    return _lin(w, "output_layer", f).view(B, N, action_size)


def quantile_huber(q_targets, q_expected, taus, k=1.0):
    """agent.py:406-412: q_targets (B, N'), q_expected (B, N), taus (B, N, 1)."""
    td = q_targets.unsqueeze(1) - q_expected.unsqueeze(-1)
    h = torch.where(td.abs() <= k, 0.5 * td.pow(2), k * (td.abs() - 0.5 * k))
    ql = (taus - (td.detach() < 0).float()).abs() * h / k
    return ql.sum(dim=1).mean(dim=1).mean()


def clip_(grads, max_norm):
    total = torch.norm(torch.stack([torch.norm(g, 2.0) for g in grads]), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return float(total)


class Adam:
    """torch.optim.Adam(lr) defaults: betas (0.9, 0.999), eps 1e-8, no weight decay."""

    def __init__(self, names, lr=1e-4):
        self.names, self.lr, self.t = names, lr, 0
        self.m, self.v = {}, {}

    def step(self, w, grads):
        self.t += 1
        b1, b2, eps = 0.9, 0.999, 1e-8
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        for n, g in zip(self.names, grads):
            m = self.m.setdefault(n, torch.zeros_like(g))
            v = self.v.setdefault(n, torch.zeros_like(g))
            m.lerp_(g, 1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
            w[n].data.addcdiv_(m, denom, value=-self.lr / bc1)


def _leaf(sd):
    return {k: torch.tensor(np.asarray(v), dtype=torch.float32).requires_grad_(True) for k, v in sd.items()}


class ACIQNRef:
    """State of an AC-IQN agent on the CPU: local/target actor+critic weights and two Adams."""

    def __init__(self, actor_sd, critic_sd, lr=1e-4, gamma=0.99):
        self.actor, self.critic = _leaf(actor_sd), _leaf(critic_sd)
        self.t_actor = {k: v.detach().clone() for k, v in self.actor.items()}
        self.t_critic = {k: v.detach().clone() for k, v in self.critic.items()}
        self.aopt = Adam(list(self.actor), lr)
        self.copt = Adam(list(self.critic), lr)
        self.gamma = gamma

    def train(self, s, a, r, ns, d, taus):
        """agent.py:386-432 with the three tau draws supplied. r, d: (B, 1)."""
        with torch.no_grad():
            na = actor_forward(self.t_actor, ns)
            qn = critic_forward(self.t_critic, ns, na, taus[0])
        qt = r + self.gamma * qn * (1.0 - d)
        qe = critic_forward(self.critic, s, a, taus[1])
        closs = quantile_huber(qt, qe, taus[1])
        names = list(self.critic)
        g = torch.autograd.grad(closs, [self.critic[n] for n in names])
        g = [x.clone() for x in g]
        cgn = clip_(g, 0.5)
        self.copt.step(self.critic, g)
        ao = actor_forward(self.actor, s)
        aloss = -critic_forward(self.critic, s, ao, taus[2]).mean()
        an = list(self.actor)
        g = [x.clone() for x in torch.autograd.grad(aloss, [self.actor[n] for n in an])]
        agn = clip_(g, 0.5)
        self.aopt.step(self.actor, g)
        return float(closs.detach()), float(aloss.detach()), cgn, agn


class IQNRef:
    def __init__(self, sd, lr=1e-4, gamma=0.99):
        self.w = _leaf(sd)
        self.t = {k: v.detach().clone() for k, v in self.w.items()}
        self.opt = Adam(list(self.w), lr)
        self.gamma = gamma

    def train(self, s, a, r, ns, d, taus):
        """agent.py:434-476; a (B,) int64, taus (target, local)."""
        with torch.no_grad():
            qn = iqn_forward(self.t, ns, taus[0]).max(2)[0]
        qt = r + self.gamma * qn * (1.0 - d)
        B, N = taus[1].shape[0], taus[1].shape[1]
        qe = iqn_forward(self.w, s, taus[1]).gather(2, a.view(B, 1, 1).expand(B, N, 1)).squeeze(-1)
        loss = quantile_huber(qt, qe, taus[1])
        names = list(self.w)
        g = [x.clone() for x in torch.autograd.grad(loss, [self.w[n] for n in names])]
        gn = clip_(g, 0.5)
        self.opt.step(self.w, g)
        return float(loss.detach()), gn


# ---------------------------------------------------------------------------- bf16 training build
def bf16_round(x):
    """Round-to-nearest-even to bf16 and back (v_cvt_pk_bf16_f32, the training build's operand cast)."""
    return x.to(torch.bfloat16).to(x.dtype)


def _forward_bf16(w, s, a, taus, rnd, dtype):
    """The forward of critic_step_bf16 (its rounding points, see there); returns the intermediates."""
    f64 = dtype
    W = {k: torch.as_tensor(v).to(f64) for k, v in w.items()}
    s_self, s_obj, s_mask = (torch.as_tensor(x).to(f64) for x in s)
    a = torch.as_tensor(a).to(f64)
    taus = torch.as_tensor(taus).to(f64)
    B, N = taus.shape
    wc, w1, w2 = (rnd(W[p + ".weight"]) for p in ("cos_embedding", "hidden_layer", "hidden_layer_2"))
    bc, b1, b2 = (W[p + ".bias"] for p in ("cos_embedding", "hidden_layer", "hidden_layer_2"))
    wo, bo = W["output_layer.weight"][0], W["output_layer.bias"][0]
    # encoders: the launch's own f32 arithmetic, op for op (stage_fg: d = ((0 + w0 x0) + w1 x1) + ...,
    # relu(d + b); no FMA), so F and G are bit-identical to the kernel's before F's bf16 rounding
    def enc32(wk, bk, x):
        w32, b32, x32 = W[wk].float(), W[bk].float(), x.float()
        acc = torch.zeros(x32.shape[:-1] + (w32.shape[0],), dtype=torch.float32)
        for i in range(w32.shape[1]):
            acc = acc + w32[:, i] * x32[..., i:i + 1]
        return torch.relu(acc + b32).to(f64)
    if rnd is bf16_round:
        f_self = enc32("self_encoder.0.weight", "self_encoder.0.bias", s_self)
        f_obj = enc32("object_encoder.0.weight", "object_encoder.0.bias", s_obj)
        G = enc32("action_encoder.0.weight", "action_encoder.0.bias", a)                       # (B,128)
    else:
        f_self = torch.relu(s_self @ W["self_encoder.0.weight"].T + W["self_encoder.0.bias"])
        f_obj = torch.relu(s_obj @ W["object_encoder.0.weight"].T + W["object_encoder.0.bias"])
        G = torch.relu(a @ W["action_encoder.0.weight"].T + W["action_encoder.0.bias"])
    f_obj = f_obj * (s_mask >= 0.5).to(f64).unsqueeze(-1)                                      # (B,5,40)
    Fb = rnd(torch.cat((f_self, f_obj.reshape(B, 200)), 1))                                    # (B,256)
    if rnd is bf16_round:
        # the bf16 build's cosine (asvrl_mfma.h cos_pi_k_tau): v_cos_f32 of the f32 revolution count
        # tau * (k / 2), i.e. cos(2 pi f32(tau k / 2)), evaluated here in f64
        rev = taus.float().reshape(B * N, 1) * (0.5 * torch.arange(64, dtype=torch.float32))
        cos = rnd(torch.cos(2 * math.pi * rev.double()).to(f64))
    else:
        pis = torch.tensor([np.pi * i for i in range(64)], dtype=torch.float32).to(f64)   # AC_IQN_model.py:389
        cos = torch.cos(taus.reshape(B * N, 1) * pis)                                           # (R,64)
    Fr = Fb.repeat_interleave(N, 0)
    Gr = G.repeat_interleave(N, 0)
    c = torch.relu(cos @ wc.T + bc)
    x = rnd(Fr * c)
    h1 = torch.relu(x @ w1.T + b1)
    h1g = rnd(h1 * Gr)
    h2 = torch.relu(h1g @ w2.T + b2)
    q = (h2 @ wo + bo).view(B, N)
    return dict(W=W, s_self=s_self, s_obj=s_obj, a=a, taus=taus, B=B, N=N, wc=wc, w1=w1, w2=w2, wo=wo, bo=bo, G=G,
                Fb=Fb, cos=cos, Fr=Fr, Gr=Gr, c=c, x=x, h1=h1, h1g=h1g, h2=h2, q=q)


def critic_forward_bf16(w, s, a, taus, rnd=bf16_round, dtype=torch.float64):
    """The critic's forward (AC_IQN_model.py:410-480) with the bf16 training build's rounding points (see
    critic_step_bf16) -- those of the target critic's forward pass inside the update launch
    (asvrl_critic_train_fused_tq: asvrl_critic_tile.h critic_tile<MODE_FWD>, which forms F, G, cos, x, h1g and q
    exactly as the update's forward does). Returns q (B, N) in `dtype`."""
    return _forward_bf16(w, s, a, taus, rnd, dtype)["q"]


def critic_step_bf16(w, s, a, q_next, r, d, taus, gamma=0.99, kappa=1.0, rnd=bf16_round, dtype=torch.float64):
    """agent.py:395-414's critic gradients (AC_IQN_model.py:284-308,410-480 forward, quantile-Huber
    agent.py:701-707, backward) restated with the rounding points of the bf16 training build's ONE fused
    launch, critic_fused_kernel<N, false> (asvrl_critic_fused.hip), at which every MFMA operand is bf16 and
    every accumulation f32 -- here f64, so only the rounding points are emulated:

      weights   Wc, W1, W2 as bf16 images (biases, wo, the encoders f32; bias = the accumulator's start)
      forward   F = bf16(relu(enc(s)))  (masked objects 0), G = relu(enc_a(a)) f32, cos = bf16(cos(tau pi k)),
                c = relu(bc + Wc cos), x = bf16(F c), h1 = relu(b1 + W1 x), h1g = bf16(h1 G),
                h2 = relu(b2 + W2 h1g), q = wo . h2 + bo (h2 f32)
      loss      the quantile-Huber terms against r + gamma q_next (1 - d), dq = dL/dq
      backward  dz2 = bf16(dq wo 1[h2 > 0]); d wo = sum dq bf16(h2); dh1g = W2^T dz2;
                dz1 = bf16(dh1g G 1[h1 > 0]); dG = sum_tau dh1g bf16(h1); dx = W1^T dz1;
                dF = sum_tau dx c; dzc = bf16(dx F 1[c > 0]); dW = dZ^T X of the bf16 images
      encoders  dzF = dF 1[F > 0], dzG = dG 1[G > 0] (f32) into the encoders' weight / bias sums

    w: critic state_dict (f32 tensors, reference key names); s = (self (B,7), objects (B,5,5), mask (B,5));
    a (B,2); q_next (B,N') the target quantiles the launch read; r, d (B,); taus (B,N). rnd=identity
    reduces this to the plain f64 critic step (pinned to torch autograd on the reference's own batch by
    tests/test_bf16_oracle_cpu.py). dtype=torch.float32 evaluates the same rounding points with f32
    arithmetic everywhere else (CPU summation orders): the spread between the two evaluations is the
    noise floor any f32 implementation of these rounding points shows (tests/test_critic_bf16_oracle_gpu.py).
    Returns (loss, {parameter name: gradient}) in `dtype`."""
    f64 = dtype
    fw = _forward_bf16(w, s, a, taus, rnd, dtype)
    W, s_self, s_obj, a, taus, B, N = (fw[k] for k in ("W", "s_self", "s_obj", "a", "taus", "B", "N"))
    wc, w1, w2, wo, bo, G, Fb, cos, Fr, Gr = (fw[k] for k in ("wc", "w1", "w2", "wo", "bo", "G", "Fb", "cos", "Fr", "Gr"))
    c, x, h1, h1g, h2, q = (fw[k] for k in ("c", "x", "h1", "h1g", "h2", "q"))
    q_next = torch.as_tensor(q_next).to(f64)
    r, d = (torch.as_tensor(v).to(f64) for v in (r, d))
    Np = q_next.shape[1]
    # quantile-Huber (agent.py:399-412): L = mean_b mean_j sum_i |tau_i - 1[delta < 0]| H(delta) / kappa
    qt = r.view(B, 1) + gamma * q_next * (1.0 - d.view(B, 1))
    delta = qt.view(B, 1, Np) - q.view(B, N, 1)
    quad = delta.abs() <= kappa
    hub = torch.where(quad, 0.5 * delta * delta, kappa * (delta.abs() - 0.5 * kappa))
    wgt = torch.where(delta < 0, 1.0 - taus.view(B, N, 1), taus.view(B, N, 1))
    loss = (wgt * hub).sum() / (kappa * B * Np)
    dH = torch.where(quad, delta, kappa * torch.sign(delta))
    dq = (-(wgt * dH).sum(2) / (kappa * B * Np)).reshape(B * N)
    # backward
    h2b = rnd(h2)
    dz2 = rnd(torch.where(h2b > 0, dq.view(-1, 1) * wo.view(1, -1), torch.zeros_like(h2)))
    g = {"output_layer.weight": (dq @ h2b).view(1, -1), "output_layer.bias": dq.sum().view(1)}
    g["hidden_layer_2.weight"], g["hidden_layer_2.bias"] = dz2.T @ h1g, dz2.sum(0)
    dh1g = dz2 @ w2
    h1b = rnd(h1)
    dz1 = rnd(torch.where(h1b > 0, dh1g * Gr, torch.zeros_like(h1)))
    dG = (dh1g * h1b).view(B, N, -1).sum(1)
    g["hidden_layer.weight"], g["hidden_layer.bias"] = dz1.T @ x, dz1.sum(0)
    dx = dz1 @ w1
    dF = (dx * c).view(B, N, -1).sum(1)
    dzc = rnd(torch.where(c > 0, dx * Fr, torch.zeros_like(c)))
    g["cos_embedding.weight"], g["cos_embedding.bias"] = dzc.T @ cos, dzc.sum(0)
    dzF = torch.where(Fb > 0, dF, torch.zeros_like(dF))
    dzG = torch.where(G > 0, dG, torch.zeros_like(dG))
    g["self_encoder.0.weight"], g["self_encoder.0.bias"] = dzF[:, :56].T @ s_self, dzF[:, :56].sum(0)
    dzo = dzF[:, 56:].reshape(B, 5, 40)
    g["object_encoder.0.weight"] = torch.einsum("bof,boi->fi", dzo, s_obj)
    g["object_encoder.0.bias"] = dzo.sum((0, 1))
    g["action_encoder.0.weight"], g["action_encoder.0.bias"] = dzG.T @ a, dzG.sum(0)
    return float(loss), g


# ---------------------------------------------------------------------------- Rainbow / C51
def _noisy(w, p, x, training=True):
    if training:
        W = w[p + ".weight_mu"] + w[p + ".weight_sigma"] * w[p + ".weight_epsilon"]
        b = w[p + ".bias_mu"] + w[p + ".bias_sigma"] * w[p + ".bias_epsilon"]
    else:
        W, b = w[p + ".weight_mu"], w[p + ".bias_mu"]
    return F.linear(x, W, b)


def rainbow_forward(w, s, atoms=51, action_size=25, obj_feat=8, log=False):
    f = _features(w, *s, obj_feat=obj_feat)
    v = _noisy(w, "output_layer_v", torch.relu(_noisy(w, "hidden_layer_v_2", torch.relu(_noisy(w, "hidden_layer_v", f)))))
    a = _noisy(w, "output_layer_a", torch.relu(_noisy(w, "hidden_layer_a_2", torch.relu(_noisy(w, "hidden_layer_a", f)))))
    v, a = v.view(-1, 1, atoms), a.view(-1, action_size, atoms)
    q = v + a - a.mean(1, keepdim=True)
    return F.log_softmax(q, dim=2) if log else F.softmax(q, dim=2)


def c51_target(pns_a, returns, nonterminal, support, gamma_n, vmin=-1.0, vmax=1.0):
    """agent.py:616-631 in numpy f32, accumulating lower masses then upper masses atom by atom."""
    p = np.asarray(pns_a, np.float32)
    B, A = p.shape
    R = np.asarray(returns, np.float32).reshape(B)
    nt = np.asarray(nonterminal, np.float32).reshape(B)
    z = np.asarray(support, np.float32)
    g = np.float32(gamma_n)
    dz = np.float32((vmax - vmin) / (A - 1))
    tz = np.clip(R[:, None] + (nt * g)[:, None] * z[None, :], np.float32(vmin), np.float32(vmax)).astype(np.float32)
    b = ((tz - np.float32(vmin)) / dz).astype(np.float32)
    l, u = np.floor(b).astype(np.int64), np.ceil(b).astype(np.int64)
    l[(u > 0) & (l == u)] -= 1
    u[(l < A - 1) & (l == u)] += 1
    m = np.zeros((B, A), np.float32)
    rows = np.arange(B)
    lo = (p * (u.astype(np.float32) - b)).astype(np.float32)
    hi = (p * (b - l.astype(np.float32))).astype(np.float32)
    for j in range(A):
        m[rows, l[:, j]] += lo[:, j]
    for j in range(A):
        m[rows, u[:, j]] += hi[:, j]
    return m


# ---------------------------------------------------------------------------------------------------
# Synthetic Rainbow_Policy state (full dims) reproducible bit for bit from numpy alone: the capture of
# the reference's train_Rainbow at the network size the kernels take (tools/capture_oracle.py
# capture_rainbow_full -> tests/golden/learn_rainbow_full.npz) stores only this generator's seed, not
# the 540k parameters. Layout follows Rainbow_model.py:17-139 (NoisyLinear: weight/bias mu, sigma and
# the factorised epsilon = f(eps_out) f(eps_in)^T, f(x) = sign(x) sqrt|x|).
RAINBOW_NOISY = (("hidden_layer_v", 256, 128), ("hidden_layer_v_2", 128, 128), ("output_layer_v", 128, 51),
                 ("hidden_layer_a", 256, 128), ("hidden_layer_a_2", 128, 128), ("output_layer_a", 128, 25 * 51))


def scaled_noise(x):
    """NoisyLinear._scale_noise (Rainbow_model.py:35-37) on given normals, f32."""
    x = np.asarray(x, np.float32)
    return (np.sign(x) * np.sqrt(np.abs(x))).astype(np.float32)


def noisy_epsilon(eps_in, eps_out):
    """reset_noise's buffers (Rainbow_model.py:39-43): weight eps = eps_out ger eps_in (one f32 product
    per element, as torch.ger), bias eps = eps_out."""
    return np.outer(eps_out, eps_in).astype(np.float32), np.asarray(eps_out, np.float32).copy()


def synthetic_rainbow_state(seed, std_init=0.05):
    """{state_dict key: f32 array} of a default-dims Rainbow_Policy (self 7 -> 56, objects 5 x (5 -> 40),
    dueling heads 256 -> 128 -> 128 -> 51 / 25 x 51): mu ~ U(-1/sqrt(in), 1/sqrt(in)) and the encoders
    likewise, sigma as NoisyLinear.reset_parameters (std_init / sqrt(fan)), epsilon from N(0, 1) draws."""
    rs = np.random.RandomState(seed)
    sd = {}
    for name, fin, fout in (("self_encoder.0", 7, 56), ("object_encoder.0", 5, 40)):
        r = 1.0 / math.sqrt(fin)
        sd[name + ".weight"] = rs.uniform(-r, r, (fout, fin)).astype(np.float32)
        sd[name + ".bias"] = rs.uniform(-r, r, fout).astype(np.float32)
    for name, fin, fout in RAINBOW_NOISY:
        r = 1.0 / math.sqrt(fin)
        sd[name + ".weight_mu"] = rs.uniform(-r, r, (fout, fin)).astype(np.float32)
        sd[name + ".weight_sigma"] = np.full((fout, fin), std_init / math.sqrt(fin), np.float32)
        sd[name + ".bias_mu"] = rs.uniform(-r, r, fout).astype(np.float32)
        sd[name + ".bias_sigma"] = np.full(fout, std_init / math.sqrt(fout), np.float32)
        we, be = noisy_epsilon(scaled_noise(rs.standard_normal(fin)), scaled_noise(rs.standard_normal(fout)))
        sd[name + ".weight_epsilon"], sd[name + ".bias_epsilon"] = we, be
    return sd
