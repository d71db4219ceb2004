"""Rainbow (dueling NoisyNet C51) act and train_Rainbow with the head and the noisy weights on
gfx950 kernels (asvrl_rainbow.hip); the layer GEMMs stay hipBLASLt GEMMs through torch.

Per learn step (agent.py:597-641), on PER rows [B][88] (obs | n-th next obs | action | R | nonterminal |
weight):
  online W = mu + sigma * eps, composed once per iteration     asvrl_noisy_compose (in act)
  logits v, a of s (with grad) and of s_{t+n}                    torch GEMMs (fp32)
  double-Q argmax over s_{t+n} with the online head              asvrl_rainbow_act (no exploration)
  target reset_noise() + compose                                 asvrl_noisy_reset (one launch)
  target logits of s_{t+n}, p(s_{t+n}, a*)                       torch GEMMs, asvrl_rainbow_pick
  projection m                                                   asvrl_c51_project (bit-exact)
  per-sample loss and d mean(w loss) / d(v, a)                   asvrl_rainbow_loss
  backward through the GEMMs                                     torch.autograd.backward([v, a], [dv, da])
  dmu = dW, dsigma = dW * eps                                    asvrl_noisy_compose(backward)
  clip + Adam                                                    asvrl_adam_clip
Act (agent.py:308-324) on every robot: the same composed online weights, logits, asvrl_rainbow_act
with epsilon-greedy on the device step counter.

The online net's noise is never resampled during training, as in the reference (its reset_noise is
only called on the target, agent.py:610). The target noise comes from Philox instead of torch.randn.
"""
import ctypes as C
import os

import torch
import torch.nn.functional as F

from . import _abi
from .learn_ops import c51_project
from .splitk_linear import SPLITK_MIN_ROWS, _SplitKLinear, _SplitKLinearReLU

NOISY = ("hidden_layer_v", "hidden_layer_v_2", "output_layer_v", "hidden_layer_a", "hidden_layer_a_2",
         "output_layer_a")
ATOMS, ACTIONS = 51, 25


class NoisyPack:
    """Composed NoisyLinear weights of one Rainbow_Policy in one flat buffer (views W[name], b[name]).
    Build it after anything that re-points the parameters (FusedAdam)."""

    def __init__(self, net):
        self.net = net
        layers = [getattr(net, n) for n in NOISY]
        dev = layers[0].weight_mu.device
        sizes = []
        for L in layers:
            sizes += [L.weight_mu.numel(), L.bias_mu.numel()]
        self.flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        s = _abi.AsvNoisySegs()
        s.n = 2 * len(layers)
        k = 0
        for L in layers:
            for mu, sig, eps in ((L.weight_mu, L.weight_sigma, L.weight_epsilon),
                                 (L.bias_mu, L.bias_sigma, L.bias_epsilon)):
                n = mu.numel()
                view = self.flat[off:off + n].view_as(mu)
                self.views.append(view)
                s.off[k] = off
                seg = s.seg[k]
                seg.mu, seg.sigma, seg.eps, seg.out = mu.data_ptr(), sig.data_ptr(), eps.data_ptr(), view.data_ptr()
                off += n
                k += 1
        s.off[k] = off
        self.segs = s
        self.layers = layers
        self.in_f = (C.c_int32 * len(layers))(*[L.in_features for L in layers])     # host arrays
        self.out_f = (C.c_int32 * len(layers))(*[L.out_features for L in layers])

    def weights(self, detach_grad=False):
        """{layer: (W, b)}; detach_grad: fresh leaf tensors (same storage) that collect dW, db."""
        ts = [v.detach().requires_grad_(True) for v in self.views] if detach_grad else self.views
        return {n: (ts[2 * j], ts[2 * j + 1]) for j, n in enumerate(NOISY)}, ts

    def compose(self, stream=None):
        _abi.check(_abi.lib().asvrl_noisy_compose(C.byref(self.segs), 0, _abi.stream_ptr(stream)),
                   "asvrl_noisy_compose")

    def reset(self, seed, counter_dev, stream=None):
        """reset_noise() on every noisy layer + compose, one launch."""
        _abi.check(_abi.lib().asvrl_noisy_reset(C.byref(self.segs), self.in_f, self.out_f,
                                                int(seed) & 0xFFFFFFFFFFFFFFFF, _abi.ptr(counter_dev),
                                                _abi.stream_ptr(stream)), "asvrl_noisy_reset")

    def backward(self, leaves, stream=None):
        """dmu = dW, dsigma = dW * eps into the parameters' .grad buffers (assigned)."""
        s = _abi.AsvNoisySegs()
        C.memmove(C.byref(s), C.byref(self.segs), C.sizeof(s))
        k = 0
        for L in self.layers:
            for mu, sig in ((L.weight_mu, L.weight_sigma), (L.bias_mu, L.bias_sigma)):
                g = leaves[k].grad
                if g is None:
                    g = torch.zeros_like(leaves[k])
                g = g.contiguous()
                leaves[k]._keep = g   # keep alive until the launch is queued
                seg = s.seg[k]
                seg.dout, seg.dmu, seg.dsigma = g.data_ptr(), mu.grad.data_ptr(), sig.grad.data_ptr()
                k += 1
        _abi.check(_abi.lib().asvrl_noisy_compose(C.byref(s), 1, _abi.stream_ptr(stream)), "asvrl_noisy_compose(bwd)")


_SPLITK = os.environ.get("ASVRL_RAINBOW_SPLITK", "1") != "0"
# rows per split-K group: 1024 gave the shortest Rainbow step of 256/512/1024/2048 (rocprof A/B)
_GROUP_ROWS = int(os.environ.get("ASVRL_RAINBOW_GROUP_ROWS", "1024"))


def _lin(x, w, b):
    """F.linear; with grad on a batch of >= SPLITK_MIN_ROWS rows the weight gradient is a split-K
    batched GEMM (a single hipBLASLt call at K = 8192 leaves most CUs idle: 50 us per layer)."""
    if _SPLITK and torch.is_grad_enabled() and x.shape[0] >= SPLITK_MIN_ROWS and (w.requires_grad or x.requires_grad):
        return _SplitKLinear.apply(x, w, b, _GROUP_ROWS)
    return F.linear(x, w, b)


_RELU_EPILOGUE = os.environ.get("ASVRL_RAINBOW_EPI", "1") != "0"


def _lin_relu(x, w, b):
    """relu(x W^T + b). Without grad on the device it is one hipBLASLt GEMM with the bias + ReLU
    epilogue (torch._addmm_activation) instead of a GEMM and a clamp launch (4-5 us each, 18 per
    Rainbow iteration in the act and target forwards)."""
    if _RELU_EPILOGUE and x.is_cuda and x.dim() == 2:
        if not torch.is_grad_enabled():
            return torch._addmm_activation(b, x, w.t())
        if _SPLITK and x.shape[0] >= SPLITK_MIN_ROWS:
            return _SplitKLinearReLU.apply(x, w, b, _GROUP_ROWS)
    return F.relu(_lin(x, w, b))


def logits(net, x, W):
    """Rainbow_Policy.forward up to the dueling combine (Rainbow_model.py:97-127): value (N, 51) and
    advantage (N, 25*51) logits with the composed noisy weights W. The encoders are
    encode_observation (AC_IQN_model.py:284-308) written out so their layers take _lin too."""
    x_1, x_2, x_2_mask = x
    B = x_1.shape[0]
    se, oe = net.self_encoder[0], net.object_encoder[0]
    f1 = _lin_relu(x_1, se.weight, se.bias)
    if x_2 is None:
        f2 = torch.zeros((B, net.max_object_num * net.object_feature_dimension), device=x_1.device, dtype=f1.dtype)
    else:
        f2 = _lin_relu(x_2.reshape(B * net.max_object_num, net.object_dimension), oe.weight, oe.bias)
        f2 = f2.view(B, net.max_object_num, net.object_feature_dimension)
        f2 = f2.masked_fill(x_2_mask.unsqueeze(-1) < 0.5, 0.0)
        f2 = f2.reshape(B, net.max_object_num * net.object_feature_dimension)
    f = torch.cat((f1, f2), 1)
    fv = _lin_relu(f, *W["hidden_layer_v"])
    fv = _lin_relu(fv, *W["hidden_layer_v_2"])
    v = _lin(fv, *W["output_layer_v"])
    fa = _lin_relu(f, *W["hidden_layer_a"])
    fa = _lin_relu(fa, *W["hidden_layer_a_2"])
    a = _lin(fa, *W["output_layer_a"])
    return v, a


def _split(rows):
    M = rows.shape[0]
    return rows[:, 0:7], rows[:, 7:32].reshape(M, 5, 5), rows[:, 32:37]


class FusedRainbow:
    """Packs and buffers (pointer-stable for graph replay) of the batched Rainbow path."""

    def __init__(self, local, target, B, support):
        self.local, self.target, self.B = local, target, B
        self.pack = NoisyPack(local)
        self.tpack = NoisyPack(target)
        dev = support.device
        self.support = support.float().contiguous()
        f = dict(dtype=torch.float32, device=dev)
        self.a_star = torch.zeros(B, dtype=torch.int64, device=dev)
        self.p_star = torch.zeros(B, ATOMS, **f)
        self.loss = torch.zeros(B, **f)
        self.dv = torch.zeros(B, ATOMS, **f)
        self.da = torch.zeros(B, ATOMS * ACTIONS, **f)
        self.pack.compose()
        self.tpack.compose()

    def target_changed(self):
        self.tpack.compose()

    def _head(self, v, a, **kw):
        io = _abi.AsvRainbowHeadIO()
        io.v, io.ldv, io.a, io.lda = v.data_ptr(), v.stride(0), a.data_ptr(), a.stride(0)
        io.N, io.atoms, io.actions_n = v.shape[0], ATOMS, ACTIONS
        io.support = self.support.data_ptr()
        for k, val in kw.items():
            setattr(io, k, val)
        return io

    @torch.no_grad()
    def act(self, obs_rows, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed):
        """act_rainbow for every row (training mode: noisy online weights), epsilon-greedy."""
        self.pack.compose()
        W, _ = self.pack.weights()
        v, a = logits(self.local, _split(obs_rows), W)
        io = self._head(v, a, act_out=actions64.data_ptr(), ld_act=actions64.stride(0), step_dev=step_dev.data_ptr(),
                        eps_steps_per_count=float(steps_per_count), eps_total=float(total),
                        eps_fraction=float(fraction), eps_initial=float(initial), eps_final=float(final),
                        seed=int(seed) & 0xFFFFFFFFFFFFFFFF)
        _abi.check(_abi.lib().asvrl_rainbow_act(C.byref(io), _abi.stream_ptr()), "asvrl_rainbow_act")

    def update(self, opt, grads, rows, gamma=0.99, n=3, vmin=-1.0, vmax=1.0, sync=None, max_norm=0.5, seed=0,
               counter_dev=None, compose=True):
        """train_Rainbow on PER rows; returns (per-sample loss, pre-clip grad norm). compose=False reuses
        the online weights composed by act() this iteration."""
        from .learner import clip_and_step
        B = rows.shape[0]
        if compose:
            self.pack.compose()
        W, leaves = self.pack.weights(detach_grad=True)
        grads.zero_()
        v, a = logits(self.local, _split(rows[:, 0:40]), W)
        with torch.no_grad():
            Wn, _ = self.pack.weights()
            vn, an = logits(self.local, _split(rows[:, 40:80]), Wn)
            io = self._head(vn, an, act_idx=self.a_star.data_ptr())
            _abi.check(_abi.lib().asvrl_rainbow_act(C.byref(io), _abi.stream_ptr()), "asvrl_rainbow_act")
            self.tpack.reset(seed, counter_dev)
            Wt, _ = self.tpack.weights()
            vt, at = logits(self.target, _split(rows[:, 40:80]), Wt)
            io = self._head(vt, at, act_idx=self.a_star.data_ptr(), p_out=self.p_star.data_ptr())
            _abi.check(_abi.lib().asvrl_rainbow_pick(C.byref(io), _abi.stream_ptr()), "asvrl_rainbow_pick")
            m = c51_project(self.p_star, rows[:, 82], rows[:, 83], self.support, vmin, vmax, gamma ** n)
            io = self._head(v.detach(), a.detach(), actions=rows.data_ptr() + 80 * 4, weights=rows.data_ptr() + 84 * 4,
                            ld_rd=rows.stride(0), m=m.data_ptr(), loss=self.loss.data_ptr(), dv=self.dv.data_ptr(),
                            da=self.da.data_ptr(), grad_scale=1.0 / B)
            _abi.check(_abi.lib().asvrl_rainbow_loss(C.byref(io), _abi.stream_ptr()), "asvrl_rainbow_loss")
        torch.autograd.backward([v, a], [self.dv, self.da])
        self.pack.backward(leaves)
        if sync is not None:
            sync(grads)
        gn = clip_and_step(opt, grads, max_norm)
        return self.loss, gn
