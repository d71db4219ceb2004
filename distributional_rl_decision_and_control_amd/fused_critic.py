"""Fused MFMA critic (csrc/asvrl_critic.hip) behind the AC-IQN update.

CriticPack turns a Critic's f32 weights into the bf16 A-operand fragments the kernel loads
(one 16-byte load per lane per v_mfma_f32_32x32x16_bf16), in the k order of the kernel's
register chaining: a layer fed from the previous accumulator sees its inputs in the order
16s + 8(j>>2) + 4h + (j&3) within each 32-feature block. Refreshing is one gather + cast per
matrix into preallocated buffers, so it can live inside a captured HIP graph.

ac_iqn_update_fused is learner.ac_iqn_update (agent.py:386-432) with the critic trunk --
cos embedding, both hidden layers, the output layer, the quantile-Huber loss and the whole
backward -- in two kernel launches per critic pass, the state/action encoders and the actor
on torch, and the trunk's weight gradients as split-K bf16 GEMMs over the saved activations.
"""
import contextlib
import ctypes as C

import torch

from . import _abi
from .learner import clip_and_step
from .policy.AC_IQN_model import encode_observation


def _p(t):
    return t.data_ptr() if t is not None else None

_IDX = {}


def frag_index(M, K, chained, device):
    """Flat indices into a row-major (M, K) matrix, ordered [mb][ks][lane][j]."""
    key = (M, K, chained, str(device))
    if key not in _IDX:
        mb = torch.arange(M // 32).view(-1, 1, 1, 1)
        ks = torch.arange(K // 16).view(1, -1, 1, 1)
        lane = torch.arange(64).view(1, 1, -1, 1)
        j = torch.arange(8).view(1, 1, 1, -1)
        r, h = lane & 31, lane >> 5
        row = mb * 32 + r
        col = ks * 16 + ((8 * (j >> 2) + 4 * h + (j & 3)) if chained else (8 * h + j))
        _IDX[key] = (row * K + col).reshape(-1).to(device)
    return _IDX[key]


class CriticPack:
    """bf16 fragment images of one Critic's trunk weights + pointers (AsvCriticWeights).
    operands="f32": f32 images for libasvrl_f32.so (the parity build); every launch on this pack
    goes to the library of its operand type (self.L)."""

    def __init__(self, critic, operands="bf16"):
        dev = critic.cos_embedding.weight.device
        self.critic = critic
        self.operands = operands
        self.L = _abi.lib(operands)
        bf = dict(dtype=_abi.operand_dtype(operands), device=dev)
        self.wc = torch.empty(256 * 64, **bf)
        self.w1 = torch.empty(128 * 256, **bf)
        self.w2 = torch.empty(128 * 128, **bf)
        self.w2t = torch.empty(128 * 128, **bf)
        self.w1t = torch.empty(256 * 128, **bf)
        self.idx = dict(wc=frag_index(256, 64, False, dev), w1=frag_index(128, 256, True, dev),
                        w2=frag_index(128, 128, True, dev), w2t=frag_index(128, 128, True, dev),
                        w1t=frag_index(256, 128, True, dev))
        s = _abi.AsvCriticWeights()
        s.wc_frag, s.w1_frag, s.w2_frag = self.wc.data_ptr(), self.w1.data_ptr(), self.w2.data_ptr()
        s.w2t_frag, s.w1t_frag = self.w2t.data_ptr(), self.w1t.data_ptr()
        s.bc, s.b1 = critic.cos_embedding.bias.data_ptr(), critic.hidden_layer.bias.data_ptr()
        s.b2, s.wo = critic.hidden_layer_2.bias.data_ptr(), critic.output_layer.weight.data_ptr()
        s.bo = critic.output_layer.bias.data_ptr()
        # f32 encoders, read by the kernels when given observation rows (encoders fused in the trunk)
        s.self_w, s.self_b = critic.self_encoder[0].weight.data_ptr(), critic.self_encoder[0].bias.data_ptr()
        s.obj_w, s.obj_b = critic.object_encoder[0].weight.data_ptr(), critic.object_encoder[0].bias.data_ptr()
        if hasattr(critic, "action_encoder"):
            s.ae_w, s.ae_b = critic.action_encoder[0].weight.data_ptr(), critic.action_encoder[0].bias.data_ptr()
        self.struct = s
        self.refresh()

    def adam_segments(self, opt):
        """The five trunk images as AsvPackSeg of FusedAdam `opt` (asvrl_adam_step_pack)."""
        c = self.critic
        W1, W2 = c.hidden_layer.weight, c.hidden_layer_2.weight
        return [opt.pack_seg(c.cos_embedding.weight, self.wc, K=64),
                opt.pack_seg(W1, self.w1, K=256, chained=True), opt.pack_seg(W1, self.w1t, K=128, chained=True,
                                                                            transposed=True),
                opt.pack_seg(W2, self.w2, K=128, chained=True), opt.pack_seg(W2, self.w2t, K=128, chained=True,
                                                                            transposed=True)]

    def refresh(self, stream=None):
        """Re-pack from the critic's current f32 weights: one asvrl_critic_pack launch."""
        c = self.critic
        rc = self.L.asvrl_critic_pack(_abi.ptr(c.cos_embedding.weight), _abi.ptr(c.hidden_layer.weight),
                                      _abi.ptr(c.hidden_layer_2.weight), C.byref(self.struct),
                                      _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_critic_pack", self.L)

    @torch.no_grad()
    def reference_images(self):
        """The same five images by torch gathers (frag_index), for the packing test."""
        c = self.critic
        W1, W2 = c.hidden_layer.weight, c.hidden_layer_2.weight
        out = {}
        for name, W in (("wc", c.cos_embedding.weight), ("w1", W1), ("w2", W2), ("w2t", W2.t().contiguous()),
                        ("w1t", W1.t().contiguous())):
            out[name] = torch.index_select(W.reshape(-1), 0, self.idx[name]).to(_abi.operand_dtype(self.operands))
        return out


def _io(F, G, taus, N, obs=None, act=None, xb=None, **kw):
    """AsvCriticIO for one launch; tensors become device pointers, None -> NULL. With `obs`
    (packed observation rows, any row stride) F may be None, with `act` ([B][2] view) G may be
    None: the kernels then run the encoders themselves."""
    io = _abi.AsvCriticIO()
    io.F, io.G, io.taus = _p(F), _p(G), taus.data_ptr()
    io.B, io.N = (F if F is not None else obs).shape[0], N
    if obs is not None:
        assert obs.dtype == torch.float32 and obs.stride(-1) == 1
        io.obs, io.ld_obs = obs.data_ptr(), obs.stride(0)
    if act is not None:
        assert act.dtype == torch.float32 and act.stride(-1) == 1
        io.act, io.ld_act = act.data_ptr(), act.stride(0)
    io.xb = _p(xb)
    io.Np, io.kappa, io.gamma, io.dq, io.ld_rd = kw.pop("Np", 0), kw.pop("kappa", 1.0), kw.pop("gamma", 0.0), \
        kw.pop("dq", 0.0), kw.pop("ld_rd", 1)
    io.loss_scale = kw.pop("loss_scale", 0.0)
    for k, v in kw.items():
        setattr(io, k, v.data_ptr() if v is not None else None)
    return io


def critic_forward(pack, F, G, taus, N, q=None, stream=None, obs=None, act=None):
    B = (F if F is not None else obs).shape[0]
    q = q if q is not None else torch.empty(B * N, dtype=torch.float32, device=taus.device)
    io = _io(F, G, taus, N, obs=obs, act=act, q=q)
    _abi.check(pack.L.asvrl_critic_forward(C.byref(pack.struct), C.byref(io), _abi.stream_ptr(stream)),
               "asvrl_critic_forward", pack.L)
    return q.view(B, N)


class TrainBuffers:
    """Saved activations of one TRAIN pass (operand dtype of the build, see CriticPack)."""

    def __init__(self, B, N, device, operands="bf16"):
        R = B * N
        bf = dict(dtype=_abi.operand_dtype(operands), device=device)
        self.B, self.N = B, N
        self.cos = torch.empty(R, 64, **bf)
        self.h0 = torch.empty(R, 256, **bf)
        self.dzc = torch.empty(R, 256, **bf)
        self.h1g = torch.empty(R, 128, **bf)
        self.dz1 = torch.empty(R, 128, **bf)
        self.h2 = torch.empty(R, 128, **bf)
        self.dz2 = torch.empty(R, 128, **bf)
        f = dict(dtype=torch.float32, device=device)
        self.dq = torch.empty(R, **f)
        self.row_loss = torch.empty(R, **f)
        self.q = torch.empty(R, **f)
        self.dF = torch.empty(B, 256, **f)
        self.dG = torch.empty(B, 128, **f)
        self.work_floats = max(int(_abi.lib(operands).asvrl_linear_wgrad_workspace(M, K))
                               for M, K in ((256, 64), (128, 256), (128, 128)))
        self.work = torch.empty(self.work_floats, **f)
        a = _abi.AsvCriticActs()
        a.cos, a.h0, a.dzc, a.h1g = self.cos.data_ptr(), self.h0.data_ptr(), self.dzc.data_ptr(), self.h1g.data_ptr()
        a.dz1, a.h2, a.dz2, a.dq = self.dz1.data_ptr(), self.h2.data_ptr(), self.dz2.data_ptr(), self.dq.data_ptr()
        self.struct = a


def wout_groups(B, N):
    """Partials critic_train(wout_part=...) writes (one per TRAIN workgroup)."""
    return int(_abi.lib().asvrl_critic_wout_groups(B, N))


def critic_train(pack, F, G, taus, q_targets, bufs, kappa=1.0, stream=None, q_next=None, rewards=None, dones=None,
                 gamma=0.99, dzF=None, dzG=None, with_dFdG=True, tile_loss=None, obs=None, act=None, xb=None,
                 wout_part=None):
    """TRAIN launch. Targets: q_targets (B, Np), or q_next (B, Np) with rewards/dones column
    views (stride ld) combined in the kernel. With `tile_loss` ([B*N/32] f32) the kernel writes
    per-tile loss partials (sum them, e.g. in a PartialArena) and None is returned; otherwise
    the loss row_loss.sum() / (B*Np) as a 0-d device tensor. With `wout_part` ([wout_groups(B, N)]
    [129] f32) the output layer's weight / bias gradient leaves as per-workgroup partials
    (PartialArena.tiles) and neither h2 nor dq is written."""
    B, N = (F if F is not None else obs).shape[0], bufs.N
    Np = (q_targets if q_targets is not None else q_next).shape[1]
    kw = dict(q=bufs.q, row_loss=bufs.row_loss, dzF=dzF, dzG=dzG, tile_loss=tile_loss,
              loss_scale=1.0 / float(B * Np))
    if with_dFdG:
        kw.update(dF=bufs.dF, dG=bufs.dG)
    if q_targets is not None:
        kw["q_targets"] = q_targets
    else:
        kw.update(q_next=q_next, rewards=rewards, dones=dones, ld_rd=rewards.stride(0), gamma=float(gamma))
    io = _io(F, G, taus, N, obs=obs, act=act, xb=xb, Np=Np, kappa=float(kappa), **kw)
    acts = bufs.struct
    if wout_part is not None:
        assert wout_part.numel() >= wout_groups(B, N) * 129
        acts = _abi.AsvCriticActs()
        C.memmove(C.byref(acts), C.byref(bufs.struct), C.sizeof(acts))
        acts.h2, acts.dq, acts.wout_part = None, None, wout_part.data_ptr()
    _abi.check(pack.L.asvrl_critic_train(C.byref(pack.struct), C.byref(io), C.byref(acts),
                                         _abi.stream_ptr(stream)), "asvrl_critic_train", pack.L)
    if tile_loss is not None:
        return None
    return bufs.row_loss.sum() / float(B * Np)


class fused_variant:
    """Context manager (or plain call) selecting asvrl_critic_train_fused(_tq)'s kernel where both forms take the
    shape (ABI 23, asvrl_critic_fused_variant): 4 = the one-wave-per-SIMD kernel (the default), 8 = two waves per
    SIMD (measured 11 % slower; its tests and the A/B select it). Process-wide, bf16 build."""

    def __init__(self, v, operands="bf16"):
        self.L = _abi.lib(operands)
        self.prev = int(self.L.asvrl_critic_fused_variant(int(v)))
        _abi.check(0 if self.prev >= 0 else -1, "asvrl_critic_fused_variant", self.L)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.L.asvrl_critic_fused_variant(self.prev)
        return False


def fused_groups(pack, B, N):
    """Workgroups (= partial groups) of critic_train_fused; 0 when the shape is unsupported."""
    return int(pack.L.asvrl_critic_fused_groups(B, N))


def fused_train_supported(pack, B, N):
    """asvrl_critic_train_fused's shape rule: N in (8, 16, 32), B*N a multiple of its round size."""
    rows = 32 if pack.operands == "f32" else 64
    return N in (8, 16, 32) and B > 0 and (B * N) % rows == 0


def critic_train_fused(pack, critic, taus, N, q_next, rewards, dones, gamma, obs, act, arena, dzF=None, dzG=None,
                       xb=None, tile_loss=None, kappa=1.0, q=None, row_loss=None, stream=None, encoders=False,
                       target=None):
    """asvrl_critic_train_fused: the critic step's forward, quantile-Huber loss against
    r + gamma q_next (1 - d), backward AND the trunk's weight gradients in one launch. The per-workgroup
    partials land in `arena` (PartialArena) as segments of critic's cos_embedding / hidden_layer /
    hidden_layer_2 / output_layer .grad (reduced by the arena's next flush).
    encoders=True: the launch also forms the observation / action encoders' gradients (ABI 16
    parts.enc / parts.aenc) as segments of their .grad, which must be contiguous
    [self_w | self_b | obj_w | obj_b] (FusedAdam); dzF / dzG / xb are then not needed.
    target=(target_pack, taus', obs', act'): asvrl_critic_train_fused_tq (ABI 20) -- the same launch first
    computes q_next = target_critic(obs', act', taus') for the samples each workgroup updates (the values
    critic_forward(target_pack, ...) gives) into `q_next`, then the update reads it."""
    B = obs.shape[0]
    groups = fused_groups(pack, B, N)
    assert groups > 0 and fused_train_supported(pack, B, N), (B, N)
    shapes = ((critic.cos_embedding, 256, 64), (critic.hidden_layer, 128, 256), (critic.hidden_layer_2, 128, 128),
              (critic.output_layer, 1, 128))
    regions = [arena._take(groups * (M * K + M)) for _, M, K in shapes]
    parts = _abi.AsvCriticParts()
    parts.cos_emb, parts.hidden, parts.hidden2, parts.out = (t.data_ptr() for t in regions)
    if encoders:
        se, oe, ae = critic.self_encoder[0], critic.object_encoder[0], critic.action_encoder[0]
        gs = [se.weight.grad, se.bias.grad, oe.weight.grad, oe.bias.grad]
        if not all(gs[k].data_ptr() + 4 * gs[k].numel() == gs[k + 1].data_ptr() for k in range(3)):
            raise RuntimeError("critic_train_fused(encoders=True) needs the encoder gradients contiguous (FusedAdam)")
        enc_part, ae_part = arena._take(groups * 688), arena._take(groups * 384)
        parts.enc, parts.aenc = enc_part.data_ptr(), ae_part.data_ptr()
    io = _io(None, None, taus, N, obs=obs, act=act, xb=xb, Np=N, kappa=float(kappa), q_next=q_next,
             rewards=rewards, dones=dones, ld_rd=rewards.stride(0), gamma=float(gamma), q=q, row_loss=row_loss,
             dzF=dzF, dzG=dzG, tile_loss=tile_loss, loss_scale=1.0 / float(B * N))
    if target is None:
        _abi.check(pack.L.asvrl_critic_train_fused(C.byref(pack.struct), C.byref(io), C.byref(parts),
                                                   _abi.stream_ptr(stream)), "asvrl_critic_train_fused", pack.L)
    else:
        tpack, ttaus, tobs, tact = target
        assert q_next.is_contiguous() and q_next.dtype == torch.float32
        tio = _io(None, None, ttaus, N, obs=tobs, act=tact)
        _abi.check(pack.L.asvrl_critic_train_fused_tq(C.byref(pack.struct), C.byref(io), C.byref(parts),
                                                      C.byref(tpack.struct), C.byref(tio), _abi.stream_ptr(stream)),
                   "asvrl_critic_train_fused_tq", pack.L)
    for (layer, M, K), part in zip(shapes, regions):
        arena.groups(part, groups, M, K, layer.weight.grad, layer.bias.grad)
    if encoders:
        arena._seg(enc_part, gs[0], None, groups, 688, 0, False)
        arena._seg(ae_part, ae.weight.grad, ae.bias.grad, groups, 256, 128, False)


def critic_actor_grad(pack, F, G, taus, N, q, dG=None, stream=None, w_ae=None, dA=None, tile_loss=None, obs=None,
                      act=None):
    """ACTOR launch: dq = -1/(B*N) on every row; writes dG and/or dA (with w_ae); with
    `tile_loss` ([B*N/32]) per-tile partials of the actor loss -mean(q)."""
    B = (F if F is not None else obs).shape[0]
    io = _io(F, G, taus, N, obs=obs, act=act, dq=-1.0 / float(B * N), q=q, dG=dG, w_ae=w_ae, dA=dA,
             tile_loss=tile_loss, loss_scale=-1.0 / float(B * N))
    _abi.check(pack.L.asvrl_critic_actor_grad(C.byref(pack.struct), C.byref(io), _abi.stream_ptr(stream)),
               "asvrl_critic_actor_grad", pack.L)


def linear_wgrad(dz, x, dw, db, work, accumulate=False, stream=None):
    """dw (M, K) f32 <- dz^T x, db (M,) <- dz.sum(0) with dz (R, M), x (R, K) bf16 (asvrl_linear_wgrad)."""
    R, M = dz.shape
    K = x.shape[1]
    rc = _abi.lib().asvrl_linear_wgrad(_abi.ptr(dz), dz.stride(0), _abi.ptr(x), x.stride(0), R, M, K, _abi.ptr(dw),
                                       _abi.ptr(db), int(accumulate), _abi.ptr(work), work.numel(),
                                       _abi.stream_ptr(stream))
    _abi.check(rc, "asvrl_linear_wgrad")


def linear_wgrad_vec(dq, x, dw, db, work, accumulate=False, stream=None):
    """dw (K,) <- dq^T x, db (1,) <- dq.sum() with dq (R,) f32 (any stride), x (R, K) bf16."""
    R, K = x.shape
    rc = _abi.lib().asvrl_linear_wgrad_vec(_abi.ptr(dq), dq.stride(0), _abi.ptr(x), x.stride(0), R, K, _abi.ptr(dw),
                                           _abi.ptr(db),
                                           int(accumulate), _abi.ptr(work), work.numel(), _abi.stream_ptr(stream))
    _abi.check(rc, "asvrl_linear_wgrad_vec")


class PartialArena:
    """Weight-gradient partials of several layers, reduced together by ONE asvrl_partial_sums
    launch (instead of one reduction launch per layer). Regions are handed out in call order
    from one preallocated buffer, so the pointers repeat exactly under HIP-graph replay.
    operands: the learner build whose activations it reduces (bf16 / f32, see CriticPack)."""

    def __init__(self, floats, device, operands="bf16"):
        self.L = _abi.lib(operands)
        self.dtype = _abi.operand_dtype(operands)
        self.buf = torch.empty(int(floats), dtype=torch.float32, device=device)
        self.off = 0
        self.segs = []
        self.pending = None   # inside batch(): MFMA weight-gradient layers waiting for one launch
        # flush(norm=...): per-workgroup squared-norm partials
        self.norm_parts = torch.zeros(_abi.MAX_SUM_SEGS * 1024, dtype=torch.float64, device=device)
        self.nparts = 0

    def _take(self, n):
        if self.off + n > self.buf.numel():
            raise RuntimeError("PartialArena too small")
        t = self.buf[self.off:self.off + n]
        self.off += (n + 63) // 64 * 64
        return t

    def _seg(self, part, dw, db, groups, nw, nb, accumulate, stride=0, boff=0, mode=_abi.SUM_PLAIN, norm=True):
        g = _abi.AsvPartialSum()
        g.partial, g.dw, g.db = part.data_ptr(), dw.data_ptr(), (db.data_ptr() if db is not None else None)
        g.groups, g.nw, g.nb, g.accumulate = groups, nw, nb, int(accumulate)
        g.stride, g.boff, g.mode, g.norm = stride, boff, mode, int(norm)
        self.segs.append(g)
        if len(self.segs) == _abi.MAX_SUM_SEGS:
            if self.pending is not None:   # the reduction would run before the batched launch
                raise RuntimeError("PartialArena: too many segments inside batch()")
            self.flush()

    @contextlib.contextmanager
    def batch(self, stream=None):
        """linear() / fold() calls inside the block queue their layers; on exit ONE
        asvrl_linear_wgrad_multi launch writes all their partials (bit-identical to one launch
        per layer), instead of several launches on side streams joined back."""
        assert self.pending is None, "PartialArena.batch does not nest"
        self.pending = []
        try:
            yield self
        finally:
            segs, self.pending = self.pending, None
            for i in range(0, len(segs), _abi.MAX_WGRAD_SEGS):
                chunk = segs[i:i + _abi.MAX_WGRAD_SEGS]
                arr = (_abi.AsvWgradSeg * len(chunk))(*chunk)
                groups = (C.c_int32 * len(chunk))()
                _abi.check(self.L.asvrl_linear_wgrad_multi(arr, len(chunk), groups, _abi.stream_ptr(stream)),
                           "asvrl_linear_wgrad_multi", self.L)

    def _linear_partial(self, dz, x, stream):
        R, M = dz.shape
        K = x.shape[1]
        L = self.L
        ngroups = int(L.asvrl_linear_wgrad_groups(R, M, K))
        part = self._take(ngroups * (M * K + M))
        if self.pending is not None:
            assert dz.dtype == x.dtype == self.dtype and dz.stride(1) == 1 and x.stride(1) == 1
            g = _abi.AsvWgradSeg()
            g.dz, g.ldz, g.x, g.ldx = dz.data_ptr(), dz.stride(0), x.data_ptr(), x.stride(0)
            g.R, g.M, g.K, g.partial, g.partial_floats = R, M, K, part.data_ptr(), part.numel()
            g.kind = _abi.WGRAD_MFMA
            self.pending.append(g)
            return part, ngroups, M, K
        groups = C.c_int32(0)
        _abi.check(L.asvrl_linear_wgrad_partial(_abi.ptr(dz), dz.stride(0), _abi.ptr(x), x.stride(0), R, M, K,
                                                _abi.ptr(part), part.numel(), C.byref(groups),
                                                _abi.stream_ptr(stream)), "asvrl_linear_wgrad_partial", L)
        return part, groups.value, M, K

    def linear(self, dz, x, dw, db, accumulate=False, stream=None, norm=True):
        """dw (<= M rows of K) <- dz^T x, db <- dz.sum(0); a dw / db with fewer rows than dz's M
        columns takes the leading rows (a padded 32-row output layer). norm=False: outputs that are not
        parameter gradients themselves (left out of flush(norm=...)'s squared norm)."""
        part, groups, M, K = self._linear_partial(dz, x, stream)
        assert dw.numel() % K == 0 and dw.numel() <= M * K and (db is None or db.numel() <= M)
        self._seg(part, dw, db, groups, dw.numel(), db.numel() if db is not None else M, accumulate,
                  stride=M * K + M, boff=M * K, norm=norm)

    def fold(self, dz, x, net, stream=None):
        """The observation encoders' gradients of `net` from the 256 x 32 encoder-image rows
        (dz [R][256], x [R][32] bf16), folded in the reduction itself (ASVRL_SUM_FOLD_ENCODERS)."""
        se, oe = net.self_encoder[0], net.object_encoder[0]
        gs = [se.weight.grad, se.bias.grad, oe.weight.grad, oe.bias.grad]
        contiguous = all(gs[k].data_ptr() + 4 * gs[k].numel() == gs[k + 1].data_ptr() for k in range(3))
        if not contiguous:   # separate gradient tensors: plain sum into scratch + asvrl_encoder_fold
            raise RuntimeError("PartialArena.fold needs the encoder gradients contiguous (FusedAdam / FlatGrads)")
        part, groups, M, K = self._linear_partial(dz, x, stream)
        assert (M, K) == (256, 32)
        self._seg(part, gs[0], None, groups, 688, 0, False, stride=M * K + M, boff=M * K,
                  mode=_abi.SUM_FOLD_ENCODERS)

    def _queue(self, kind, dz, ldz, x, ldx, R, M, K, part):
        g = _abi.AsvWgradSeg()
        g.dz, g.ldz, g.x, g.ldx = dz.data_ptr(), ldz, x.data_ptr(), ldx
        g.R, g.M, g.K, g.kind, g.partial, g.partial_floats = R, M, K, kind, part.data_ptr(), part.numel()
        self.pending.append(g)

    def vec(self, dq, x, dw, db, accumulate=False, stream=None):
        R, K = x.shape
        L = self.L
        ngroups = int(L.asvrl_linear_wgrad_vec_groups(R))
        part = self._take(ngroups * (K + 1))
        if self.pending is not None and K == 128:
            assert dq.dtype == torch.float32 and x.dtype == self.dtype and x.stride(1) == 1
            self._queue(_abi.WGRAD_VEC, dq, dq.stride(0), x, x.stride(0), R, 1, K, part)
            self._seg(part, dw, db, ngroups, K, 1, accumulate)
            return
        groups = C.c_int32(0)
        _abi.check(L.asvrl_linear_wgrad_vec_partial(_abi.ptr(dq), dq.stride(0), _abi.ptr(x), x.stride(0), R, K,
                                                    _abi.ptr(part), part.numel(), C.byref(groups),
                                                    _abi.stream_ptr(stream)), "asvrl_linear_wgrad_vec_partial", L)
        self._seg(part, dw, db, groups.value, K, 1, accumulate)

    def take_tiles(self, tiles, nw):
        """A region for [tiles][nw + 1] per-tile partials written by a kernel (critic_train's
        wout_part); queue its reduction with tiles() after the launch."""
        return self._take(tiles * (nw + 1))

    def tiles(self, part, tiles, dw, db, accumulate=False):
        """dw (nw) (+)= sum over tiles of part[t][0:nw], db (+)= sum of part[t][nw]."""
        self._seg(part, dw, db, tiles, dw.numel(), 1, accumulate)

    def groups(self, part, groups, M, K, dw, db, accumulate=False):
        """dw (M x K) (+)= sum over groups of part[g][0:M*K], db (M) (+)= of part[g][M*K:]: per-workgroup
        partials a kernel wrote in the [groups][M*K + M] layout (critic_train_fused); a dw / db with fewer
        rows takes the leading rows (IQN's padded 32-row output layer)."""
        assert dw.numel() % K == 0 and dw.numel() <= M * K and db.numel() <= M
        self._seg(part, dw, db, groups, dw.numel(), db.numel(), accumulate, stride=M * K + M, boff=M * K)

    def scalar(self, partials, out, accumulate=False):
        """out (1 f32) (+)= sum(partials): a scalar segment (e.g. per-tile loss partials)."""
        self._seg(partials, out, None, partials.numel(), 1, 0, accumulate, norm=False)

    def small(self, dz, x, dw, db, accumulate=False, stream=None):
        R, M = dz.shape
        K = x.shape[1]
        part = self._take(((R + 31) // 32) * (M * K + M))
        if self.pending is not None:
            assert dz.dtype == x.dtype == torch.float32 and dz.stride(1) == 1 and x.stride(1) == 1
            self._queue(_abi.WGRAD_SMALL, dz, dz.stride(0), x, x.stride(0), R, M, K, part)
            self._seg(part, dw, db, (R + 31) // 32, M * K, M, accumulate)
            return
        groups = C.c_int32(0)
        _abi.check(self.L.asvrl_small_wgrad_partial(dz.data_ptr(), dz.stride(0), x.data_ptr(), x.stride(0), R,
                                                    M, K, part.data_ptr(), part.numel(), C.byref(groups),
                                                    _abi.stream_ptr(stream)), "asvrl_small_wgrad_partial", self.L)
        self._seg(part, dw, db, groups.value, M * K, M, accumulate)

    def flush(self, stream=None, norm=None):
        """One reduction launch for the queued segments. norm: a FusedAdam whose gradients are
        exactly these segments' outputs; the launch then also leaves the squared-norm partials in
        self.norm_parts[:self.nparts] and advances its step, for norm.step_prenormed(...)."""
        if self.segs:
            arr = (_abi.AsvPartialSum * len(self.segs))(*self.segs)
            L = self.L
            if norm is not None:
                self.nparts = int(L.asvrl_partial_sums_norm_parts(arr, len(self.segs)))
                assert 1 <= self.nparts <= self.norm_parts.numel()
                _abi.check(L.asvrl_partial_sums_norm(arr, len(self.segs), _abi.ptr(self.norm_parts),
                                                     _abi.ptr(norm.step_t), _abi.stream_ptr(stream)),
                           "asvrl_partial_sums_norm", L)
            else:
                _abi.check(L.asvrl_partial_sums(arr, len(self.segs), _abi.stream_ptr(stream)), "asvrl_partial_sums",
                           L)
        elif norm is not None:
            raise RuntimeError("PartialArena.flush(norm=...) with nothing queued")
        self.segs = []
        self.off = 0


def trunk_weight_grads_into(arena, critic, bufs):
    """Queue the trunk layers' weight/bias gradients on a PartialArena (reduced at its flush)."""
    arena.linear(bufs.dzc, bufs.cos, critic.cos_embedding.weight.grad, critic.cos_embedding.bias.grad)
    arena.linear(bufs.dz1, bufs.h0, critic.hidden_layer.weight.grad, critic.hidden_layer.bias.grad)
    arena.linear(bufs.dz2, bufs.h1g, critic.hidden_layer_2.weight.grad, critic.hidden_layer_2.bias.grad)
    arena.vec(bufs.dq, bufs.h2, critic.output_layer.weight.grad, critic.output_layer.bias.grad)


def trunk_weight_grads(critic, bufs):
    """Weight/bias gradients of the fused trunk layers from the TRAIN activations: four
    asvrl_linear_wgrad launches pairs (MFMA reduction over the B*N rows + partial sum)."""
    linear_wgrad(bufs.dzc, bufs.cos, critic.cos_embedding.weight.grad, critic.cos_embedding.bias.grad, bufs.work)
    linear_wgrad(bufs.dz1, bufs.h0, critic.hidden_layer.weight.grad, critic.hidden_layer.bias.grad, bufs.work)
    linear_wgrad(bufs.dz2, bufs.h1g, critic.hidden_layer_2.weight.grad, critic.hidden_layer_2.bias.grad, bufs.work)
    linear_wgrad_vec(bufs.dq, bufs.h2, critic.output_layer.weight.grad, critic.output_layer.bias.grad, bufs.work)
