"""Rainbow (dueling NoisyNet C51) act and train_Rainbow on gfx950 kernels, no torch GEMM or autograd:
the whole network + head of act, of the two s_{t+n} passes and of the training pass (forward, loss,
backward) as one kernel per 32-row tile each (asvrl_rainbow_net.hip), the noisy weights in
asvrl_rainbow.hip, the weight gradients in asvrl_wgrad.hip.

Per learn step (agent.py:597-641), on PER rows [B][88] (obs | n-th next obs | action | R | nonterminal |
weight):
  online W = mu + sigma * eps, composed + packed once per iteration
                                                                 asvrl_noisy_compose, asvrl_rainbow_pack (in act)
  double-Q argmax over s_{t+n} with the online net               asvrl_rainbow_net_argmax (one launch)
  target reset_noise() + compose, packed                         asvrl_noisy_reset, asvrl_rainbow_pack
  p(s_{t+n}, a*) of the target net                               asvrl_rainbow_net_pick (one launch)
  projection m                                                   asvrl_c51_project (bit-exact)
  forward of s saving the activations, per-sample loss, backward to the encoders' pre-activations
                                                                 asvrl_rainbow_net_train (one launch)
  weight gradients of the six layers + the encoder fold          ONE asvrl_linear_wgrad_multi, ONE
                                                                 asvrl_partial_sums (into the composed-
                                                                 weight gradient buffer)
  dmu = dW, dsigma = dW * eps                                    asvrl_noisy_compose(backward)
  clip + Adam                                                    asvrl_adam_clip
Act (agent.py:308-324) on every robot: the same composed online weights, asvrl_rainbow_net_act
(network, head, epsilon-greedy on the device step counter) in one launch.
operands: the network kernel's MFMA operands, "bf16" (the training path) or "f32" (libasvrl_f32.so,
the parity build).

The online net's noise is never resampled during training, as in the reference (its reset_noise is
only called on the target, agent.py:610). The target noise comes from Philox instead of torch.randn.
"""
import ctypes as C

import torch

from . import _abi
from .fused_critic import PartialArena
from .learn_ops import c51_project

NOISY = ("hidden_layer_v", "hidden_layer_v_2", "output_layer_v", "hidden_layer_a", "hidden_layer_a_2",
         "output_layer_a")
ATOMS, ACTIONS = 51, 25


def supported(net, B):
    """The Rainbow kernels' network shape (Rainbow_Policy defaults: 256 concatenated features, 128 hidden,
    25 actions x 51 atoms, encoders 7 -> 56 and 5 x (5 -> 40)) and a batch of whole 32-row tiles."""
    return (net.concat_feature_dimension == 256 and net.hidden_dimension == 128 and net.action_size == ACTIONS
            and net.atoms == ATOMS and net.self_dimension == 7 and net.object_dimension == 5
            and net.max_object_num == 5 and net.self_feature_dimension == 56 and net.object_feature_dimension == 40
            and B > 0 and B % 32 == 0)


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

    def grad_buffer(self):
        """A flat buffer shaped like the composed weights for their gradient: {layer: (dW, db)} views."""
        if not hasattr(self, "dflat"):
            self.dflat = torch.zeros_like(self.flat)
            self.dviews = [self.dflat[(v.data_ptr() - self.flat.data_ptr()) // 4:][:v.numel()].view_as(v)
                           for v in self.views]
        return {n: (self.dviews[2 * j], self.dviews[2 * j + 1]) for j, n in enumerate(NOISY)}

    def backward(self, leaves, stream=None, sq_parts=None):
        """dmu = dW, dsigma = dW * eps into the parameters' .grad buffers (assigned); dW from the leaves'
        .grad (autograd) or, with leaves=None, from self.dviews (the gradient buffer grad_buffer() made).
        sq_parts (f64 device view): the written gradients' squared-norm partials go there (ABI 26); returns
        their count (0 without sq_parts)."""
        s = _abi.AsvNoisySegs()
        C.memmove(C.byref(s), C.byref(self.segs), C.sizeof(s))
        k = 0
        for L in self.layers:
            for mu, sig in ((L.weight_mu, L.weight_sigma), (L.bias_mu, L.bias_sigma)):
                if leaves is None:
                    g = self.dviews[k]
                else:
                    g = leaves[k].grad
                    if g is None:
                        g = torch.zeros_like(leaves[k])
                    g = g.contiguous()
                    leaves[k]._keep = g   # keep alive until the launch is queued
                seg = s.seg[k]
                seg.dout, seg.dmu, seg.dsigma = g.data_ptr(), mu.grad.data_ptr(), sig.grad.data_ptr()
                k += 1
        if sq_parts is not None:
            n = int(_abi.lib().asvrl_noisy_backward_norm_parts(C.byref(s)))
            assert 0 < n <= sq_parts.numel()
            _abi.check(_abi.lib().asvrl_noisy_backward_norm(C.byref(s), _abi.ptr(sq_parts), _abi.stream_ptr(stream)),
                       "asvrl_noisy_backward_norm")
            return n
        _abi.check(_abi.lib().asvrl_noisy_compose(C.byref(s), 1, _abi.stream_ptr(stream)), "asvrl_noisy_compose(bwd)")
        return 0


IMG_SIZES = {"enc": 256 * 32, "v1": 128 * 256, "a1": 128 * 256, "v2": 128 * 128, "a2": 128 * 128, "vo": 64 * 128,
             "mo": 64 * 128, "ao": 25 * 64 * 128}
IMGT_SIZES = {"vot": 128 * 64, "mot": 128 * 64, "aot": 25 * 128 * 64, "v2t": 128 * 128, "a2t": 128 * 128,
              "v1t": 256 * 128, "a1t": 256 * 128}
BIAS_SIZES = {"b_enc": 256, "b_v1p": 128, "b_a1p": 128, "b_v2p": 128, "b_a2p": 128, "b_vop": 64, "b_mop": 64,
              "b_aop": 25 * 64}


class RainbowNetImage:
    """Fragment images of one Rainbow_Policy for asvrl_rainbow_net_*: the encoders and the composed noisy
    layers of `noisy` (a NoisyPack of the same net), packed by refresh() (asvrl_rainbow_pack)."""

    def __init__(self, net, noisy, operands="bf16", train=False):
        self.L = _abi.lib(operands)
        dev = noisy.flat.device
        sizes = dict(IMG_SIZES, **(IMGT_SIZES if train else {}))
        self.img = torch.zeros(sum(sizes.values()), dtype=_abi.operand_dtype(operands), device=dev)
        self.bias = torch.zeros(sum(BIAS_SIZES.values()), dtype=torch.float32, device=dev)
        st = _abi.AsvRainbowImg()
        off = 0
        for n, k in sizes.items():
            setattr(st, n, self.img[off:off + k].data_ptr())
            off += k
        off = 0
        for n, k in BIAS_SIZES.items():
            setattr(st, n, self.bias[off:off + k].data_ptr())
            off += k
        self.struct = st
        W, _ = noisy.weights()
        se, oe = net.self_encoder[0], net.object_encoder[0]
        src = _abi.AsvRainbowSrc()
        src.self_w, src.self_b, src.obj_w, src.obj_b = (t.data_ptr() for t in (se.weight, se.bias, oe.weight, oe.bias))
        for key, name in (("v1", "hidden_layer_v"), ("a1", "hidden_layer_a"), ("v2", "hidden_layer_v_2"),
                          ("a2", "hidden_layer_a_2"), ("vo", "output_layer_v"), ("ao", "output_layer_a")):
            setattr(src, "w_" + key, W[name][0].data_ptr())
            setattr(src, "b_" + key, W[name][1].data_ptr())
        self.src = src

    def refresh(self, stream=None):
        _abi.check(self.L.asvrl_rainbow_pack(C.byref(self.src), C.byref(self.struct), _abi.stream_ptr(stream)),
                   "asvrl_rainbow_pack", self.L)

    def io(self, x, support, **kw):
        assert x.dtype == torch.float32 and x.stride(-1) == 1
        io = _abi.AsvRainbowNetIO()
        io.x, io.ldx, io.N = x.data_ptr(), x.stride(0), x.shape[0]
        io.support = support.data_ptr()
        for k, v in kw.items():
            setattr(io, k, v)
        return io

    def run(self, fn, io, stream=None):
        _abi.check(getattr(self.L, fn)(C.byref(self.struct), C.byref(io), _abi.stream_ptr(stream)), fn, self.L)


class FusedRainbow:
    """Packs and buffers (pointer-stable for graph replay) of the batched Rainbow path."""

    def __init__(self, local, target, B, support, operands="bf16"):
        self.local, self.target, self.B = local, target, B
        self.pack = NoisyPack(local)
        self.tpack = NoisyPack(target)
        self.img = RainbowNetImage(local, self.pack, operands, train=True)
        self.timg = RainbowNetImage(target, self.tpack, operands)
        dev = support.device
        self.support = support.float().contiguous()
        # the training pass's saved activations and pre-activation gradients (operand type)
        od = dict(dtype=_abi.operand_dtype(operands), device=dev)
        self.acts = {n: torch.zeros(B, k, **od) for n, k in (("xb", 32), ("f", 256), ("hv1", 128), ("ha1", 128),
                                                              ("hv2", 128), ("ha2", 128), ("dzv", 64), ("dza", 1280),
                                                              ("dz2v", 128), ("dz2a", 128), ("dz1v", 128),
                                                              ("dz1a", 128), ("dzf", 256))}
        self.arena = PartialArena(48 << 20, dev, operands)
        self.dW = self.pack.grad_buffer()
        f = dict(dtype=torch.float32, device=dev)
        self.a_star = torch.zeros(B, dtype=torch.int64, device=dev)
        self.p_star = torch.zeros(B, ATOMS, **f)
        self.loss = torch.zeros(B, **f)
        self.pack.compose()
        self.tpack.compose()
        self.img.refresh()
        self.timg.refresh()

    def target_changed(self):
        self.tpack.compose()
        self.timg.refresh()

    @torch.no_grad()
    def act(self, obs_rows, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed):
        """act_rainbow for every row (training mode: noisy online weights), epsilon-greedy."""
        self.pack.compose()
        self.img.refresh()
        io = self.img.io(obs_rows, self.support, act_out=actions64.data_ptr(), ld_act=actions64.stride(0),
                         step_dev=step_dev.data_ptr(), eps_steps_per_count=float(steps_per_count),
                         eps_total=float(total), eps_fraction=float(fraction), eps_initial=float(initial),
                         eps_final=float(final), seed=int(seed) & 0xFFFFFFFFFFFFFFFF)
        self.img.run("asvrl_rainbow_net_act", io)

    def update(self, opt, grads, rows, gamma=0.99, n=3, vmin=-1.0, vmax=1.0, sync=None, max_norm=0.5, seed=0,
               counter_dev=None, compose=True, reset_target=True):
        """train_Rainbow on PER rows; returns (per-sample loss, pre-clip grad norm). compose=False reuses
        the online weights composed by act() this iteration. reset_target=False keeps the target's noise
        buffers as they are (composed from them) instead of reset_noise() from Philox: the parity tests
        inject the noise the reference drew."""
        from .learner import FusedAdam, clip_and_step
        B = rows.shape[0]
        if compose:
            self.pack.compose()
            self.img.refresh()
        ns_rows = rows[:, 40:80]
        # double-Q argmax over s_{t+n} with the online net, then p(s_{t+n}, a*) of the target net with
        # fresh target noise (agent.py:605-612)
        self.img.run("asvrl_rainbow_net_argmax", self.img.io(ns_rows, self.support, act_idx=self.a_star.data_ptr()))
        if reset_target:
            self.tpack.reset(seed, counter_dev)
        else:
            self.tpack.compose()
        self.timg.refresh()
        self.timg.run("asvrl_rainbow_net_pick", self.timg.io(ns_rows, self.support, act_idx=self.a_star.data_ptr(),
                                                               p_out=self.p_star.data_ptr()))
        with torch.no_grad():
            m = c51_project(self.p_star, rows[:, 82], rows[:, 83], self.support, vmin, vmax, gamma ** n)
        # forward of s saving the activations, loss, backward to the encoders (agent.py:613-636)
        A = self.acts
        io = self.img.io(rows[:, 0:40], self.support, actions=rows.data_ptr() + 80 * 4,
                         weights=rows.data_ptr() + 84 * 4, ld_rd=rows.stride(0), m=m.data_ptr(), grad_scale=1.0 / B,
                         loss=self.loss.data_ptr(), **{k: t.data_ptr() for k, t in A.items()})
        self.img.run("asvrl_rainbow_net_train", io)
        # the six layers' weight gradients (into the composed-weight gradient buffer) and the encoder
        # fold in one launch, one reduction, then dmu = dW, dsigma = dW eps
        arena, dW, net = self.arena, self.dW, self.local
        # single process with the fused optimiser: the clip norm from the reduction (the encoders' gradients) and
        # the noisy backward (every mu / sigma gradient) instead of a norm launch over the flat gradient (ABI 26)
        prenorm = sync is None and isinstance(opt, FusedAdam) and self._prenorm_covers(opt)
        with arena.batch():
            # the output layers in the kernel's (32, 128) / (128, 128) shapes: column slices of the padded
            # dz images into the leading rows of each slice of the gradient (composed-weight gradients: not in
            # the norm, their mu / sigma gradients are)
            Wv, bv = dW["output_layer_v"]
            for i in range(2):
                arena.linear(A["dzv"][:, 32 * i:32 * i + 32], A["hv2"], Wv[32 * i:32 * i + 32], bv[32 * i:32 * i + 32],
                             norm=False)
            Wa, ba = dW["output_layer_a"]
            for i in range(10):
                arena.linear(A["dza"][:, 128 * i:128 * i + 128], A["ha2"], Wa[128 * i:128 * i + 128],
                             ba[128 * i:128 * i + 128], norm=False)
            arena.linear(A["dz2v"], A["hv1"], *dW["hidden_layer_v_2"], norm=False)
            arena.linear(A["dz2a"], A["ha1"], *dW["hidden_layer_a_2"], norm=False)
            arena.linear(A["dz1v"], A["f"], *dW["hidden_layer_v"], norm=False)
            arena.linear(A["dz1a"], A["f"], *dW["hidden_layer_a"], norm=False)
            arena.fold(A["dzf"], A["xb"], net)
        if prenorm:
            assert opt.max_norm == max_norm, (opt.max_norm, max_norm)
            arena.flush(norm=opt)
            n1 = arena.nparts
            n2 = self.pack.backward(None, sq_parts=arena.norm_parts[n1:])
            return self.loss, opt.step_prenormed(arena.norm_parts, n1 + n2)
        arena.flush()
        self.pack.backward(None)
        if sync is not None:
            sync(grads)
        gn = clip_and_step(opt, grads, max_norm)
        return self.loss, gn

    def _prenorm_covers(self, opt):
        """True when the optimiser's parameters are exactly the encoders (the reduction's norm segments) and the
        noisy layers' mu / sigma (the noisy backward's), so the two partial sets make its whole clip norm."""
        cached = getattr(self, "_prenorm_ok", None)
        if cached is None or cached[0] is not opt:
            net = self.local
            enc = sum(p.numel() for m in (net.self_encoder, net.object_encoder) for p in m.parameters())
            noisy = sum(p.numel() for L in self.pack.layers for p in (L.weight_mu, L.weight_sigma, L.bias_mu,
                                                                     L.bias_sigma))
            cached = self._prenorm_ok = (opt, enc + noisy == opt.n)
        return cached[1]
