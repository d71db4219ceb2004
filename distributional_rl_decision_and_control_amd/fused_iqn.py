"""The IQN update (Agent.train_IQN, agent.py:434-476) and act_iqn (agent.py:227-256) on the
gfx950 kernels of csrc/asvrl_critic.hip, csrc/asvrl_mlp.hip and csrc/asvrl_wgrad.hip.

IQN_Policy (IQN_model.py:74-108) is the AC-IQN critic trunk without the action encoder and
with a 128 -> 25 output layer, so it runs on the critic kernels' IQN modes. Per step, on a
replay batch `rows` ([B][88]: obs | next obs | action | reward | done):

    target encoders(ns) + trunk, max over actions per tau -> q_next
                                                          asvrl_iqn_forward_max    (agent.py:451-452)
                                                          (bf16 build, FusedIQNState.target_in_fused: inside
                                                          the next launch, ABI 24 asvrl_iqn_train_fused_tq)
    local encoders(s) + forward, gather at a, quantile-Huber vs r + g q_next (1-d), backward,
    and the per-workgroup weight-gradient partials of the four layers
                                                          asvrl_iqn_train_fused (ONE launch, agent.py:455-468)
    encoder gradients                                     asvrl_linear_wgrad_multi (the fold image),
                                                          ONE asvrl_partial_sums_norm: every .grad
                                                          (encoders folded, the 32-row output
                                                          reduction into the 25-row layer), the
                                                          loss and the gradient norm
    clip + Adam                                           asvrl_adam_step          (agent.py:471-472)
      (with DP: asvrl_partial_sums, RCCL all-reduce, asvrl_adam_clip)
    (B*N not a multiple of the 64-row round: asvrl_iqn_train's two launches + the weight-gradient launch over the
    saved activations, the round-1 path)
    re-pack trunk and head                                asvrl_iqn_pack

The encoders run inside the trunk kernels' prologue (f32, from the parameters). act_iqn for
every robot row is one kernel (encoders, K = 32 quantile samples per state, mean over them,
argmax, epsilon-greedy on the device step counter).

Arithmetic: bf16 MFMA operands with f32 accumulation, f32 master weights / Adam.
"""
import ctypes as C

import torch

from . import _abi
from .fused_critic import CriticPack, PartialArena, TrainBuffers, fused_groups, fused_train_supported
from .fused_update import ENC_IN_KERNEL, _reduce_and_step

OBS = 40
K_ACT = 32


# the IQN step's forward / loss / backward and weight gradients in ONE launch (asvrl_iqn_train_fused)
# wherever it takes the shape (B*N a multiple of its 64-row round); otherwise asvrl_iqn_train's two
# launches + the batched weight-gradient launch over saved activations (tests toggle it)
FUSED_TRAIN = True
# the target network's max over the actions inside that launch (ABI 24, asvrl_iqn_train_fused_tq: each workgroup
# forms q_next for the samples it updates, bit-identical to asvrl_iqn_forward_max); bf16 build. The default of
# FusedIQNState.target_in_fused. Off for the batched loop, whose act pass runs beside the learner: there the longer
# update launch runs beside the act pass instead of the env step, 0.2982 -> 0.3153 ms per IQN step; on for the
# drop-in Agent (nothing beside its update; bf16 learner): 55.5 -> 54.0 us per B = 64 step (profiles/r06j_*, r06k_*)
TARGET_IN_FUSED = False


def supported(net, B, N):
    return (net.concat_feature_dimension == 256 and net.hidden_dimension == 128 and net.n == 64
            and 1 <= net.action_size <= _abi.IQN_MAX_ACTIONS and N in (8, 16, 32) and (B * N) % 32 == 0
            and net.self_dimension == 7 and net.object_dimension == 5 and net.max_object_num == 5
            and net.self_feature_dimension == 56 and net.object_feature_dimension == 40)


class IqnPack(CriticPack):
    """bf16 images of one IQN_Policy: the trunk (CriticPack's five) and the padded output head,
    one refresh launch; the observation encoders are read in f32 by the kernels themselves.
    operands="f32": the f32 images of libasvrl_f32.so (the parity build)."""

    def __init__(self, net, operands="bf16"):
        dev = net.cos_embedding.weight.device
        self.head_img = torch.zeros(_abi.IQN_MAX_ACTIONS * 128, dtype=_abi.operand_dtype(operands), device=dev)
        hd = _abi.AsvIqnHead()
        hd.wo_frag, hd.wo, hd.bo = (self.head_img.data_ptr(), net.output_layer.weight.data_ptr(),
                                    net.output_layer.bias.data_ptr())
        hd.n_actions = net.action_size
        self.head = hd
        super().__init__(net, operands)

    def adam_segments(self, opt):
        """The trunk images and the head's leading rows (the padding rows stay zero)."""
        return super().adam_segments(opt) + [opt.pack_seg(self.critic.output_layer.weight, self.head_img, K=128,
                                                          chained=True)]

    def refresh(self, stream=None):
        n = self.critic
        rc = self.L.asvrl_iqn_pack(_abi.ptr(n.cos_embedding.weight), _abi.ptr(n.hidden_layer.weight),
                                   _abi.ptr(n.hidden_layer_2.weight), _abi.ptr(n.output_layer.weight),
                                   C.byref(self.struct), C.byref(self.head), _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_iqn_pack", self.L)


def _io(F, N, obs=None, xb=None, **kw):
    """AsvIqnIO for one launch: features F [B][256], or packed observation rows `obs` (any row
    stride; the kernels run the encoders)."""
    io = _abi.AsvIqnIO()
    io.F = F.data_ptr() if F is not None else None
    io.B, io.N = (F if F is not None else obs).shape[0], N
    if obs is not None:
        assert obs.dtype == torch.float32 and obs.stride(-1) == 1
        io.obs, io.ld_obs = obs.data_ptr(), obs.stride(0)
    io.xb = xb.data_ptr() if xb is not None else None
    for k in ("Np", "kappa", "gamma", "ld_rd", "loss_scale", "ld_act", "eps_steps_per_count", "eps_total",
              "eps_fraction", "eps_initial", "eps_final", "seed"):
        if k in kw:
            setattr(io, k, kw.pop(k))
    for k, v in kw.items():
        setattr(io, k, v.data_ptr() if v is not None else None)
    return io


def iqn_forward_max(pack, F, taus, N, q, stream=None, obs=None):
    """q[b*N + n] = max_a Q(s_b, tau_bn, a) (the target of train_IQN)."""
    io = _io(F, N, obs=obs, taus=taus, q=q)
    _abi.check(pack.L.asvrl_iqn_forward_max(C.byref(pack.struct), C.byref(pack.head), C.byref(io),
                                            _abi.stream_ptr(stream)), "asvrl_iqn_forward_max", pack.L)
    return q


def iqn_train(pack, F, taus, bufs, dz_out, q_next, actions, rewards, dones, gamma, dzF, tile_loss=None, kappa=1.0,
              q=None, stream=None, obs=None, xb=None):
    """Forward + loss + backward of the local net. actions / rewards / dones are column views of
    the replay rows (one stride). Writes bufs' activations, dz_out, dzF and, with tile_loss,
    the per-tile loss partials (loss = their sum)."""
    B, N = (F if F is not None else obs).shape[0], bufs.N
    Np = q_next.shape[1]
    assert actions.stride(0) == rewards.stride(0) == dones.stride(0)
    io = _io(F, N, obs=obs, xb=xb, taus=taus, Np=Np, kappa=float(kappa), q_next=q_next, actions=actions, rewards=rewards,
             dones=dones, ld_rd=rewards.stride(0), gamma=float(gamma), q=q, row_loss=bufs.row_loss, dzF=dzF,
             dz_out=dz_out, tile_loss=tile_loss, loss_scale=1.0 / float(B * Np))
    _abi.check(pack.L.asvrl_iqn_train(C.byref(pack.struct), C.byref(pack.head), C.byref(io),
                                      C.byref(bufs.struct), _abi.stream_ptr(stream)), "asvrl_iqn_train", pack.L)


def iqn_train_fused(pack, net, taus, N, q_next, actions, rewards, dones, gamma, obs, arena, dzF=None, xb=None,
                    tile_loss=None, kappa=1.0, q=None, row_loss=None, stream=None, encoders=False, target=None):
    """asvrl_iqn_train_fused: train_IQN's local pass (agent.py:455-468) -- forward, gather at the
    taken action, quantile-Huber loss, backward -- AND the weight gradients of the trunk and the
    output layer in one launch; the per-workgroup partials land in `arena` as segments of net's
    cos_embedding / hidden_layer / hidden_layer_2 / output_layer .grad.
    encoders=True: also the observation encoders' gradients (ABI 16 parts.enc; their .grad contiguous
    [self_w | self_b | obj_w | obj_b]); dzF / xb are then not needed.
    target=(target_pack, target_taus, next_obs): q_next is first computed inside the launch
    (asvrl_iqn_train_fused_tq) from the target network, as iqn_forward_max would."""
    B = obs.shape[0]
    groups = fused_groups(pack, B, N)
    assert groups > 0 and fused_train_supported(pack, B, N), (B, N)
    assert actions.stride(0) == rewards.stride(0) == dones.stride(0)
    shapes = ((net.cos_embedding, 256, 64), (net.hidden_layer, 128, 256), (net.hidden_layer_2, 128, 128),
              (net.output_layer, _abi.IQN_MAX_ACTIONS, 128))
    regions = [arena._take(groups * (M * K + M)) for _, M, K in shapes]
    parts = _abi.AsvCriticParts()
    parts.cos_emb, parts.hidden, parts.hidden2, parts.out = (t.data_ptr() for t in regions)
    if encoders:
        se, oe = net.self_encoder[0], net.object_encoder[0]
        gs = [se.weight.grad, se.bias.grad, oe.weight.grad, oe.bias.grad]
        if not all(gs[k].data_ptr() + 4 * gs[k].numel() == gs[k + 1].data_ptr() for k in range(3)):
            raise RuntimeError("iqn_train_fused(encoders=True) needs the encoder gradients contiguous (FusedAdam)")
        enc_part = arena._take(groups * 688)
        parts.enc = enc_part.data_ptr()
    io = _io(None, N, obs=obs, xb=xb, taus=taus, Np=N, kappa=float(kappa), q_next=q_next, actions=actions,
             rewards=rewards, dones=dones, ld_rd=rewards.stride(0), gamma=float(gamma), q=q, row_loss=row_loss,
             dzF=dzF, tile_loss=tile_loss, loss_scale=1.0 / float(B * N))
    if target is not None:
        tpack, ttaus, next_obs = target
        tio = _io(None, N, obs=next_obs, taus=ttaus)
        _abi.check(pack.L.asvrl_iqn_train_fused_tq(C.byref(pack.struct), C.byref(pack.head), C.byref(io),
                                                   C.byref(parts), C.byref(tpack.struct), C.byref(tpack.head),
                                                   C.byref(tio), _abi.stream_ptr(stream)),
                   "asvrl_iqn_train_fused_tq", pack.L)
    else:
        _abi.check(pack.L.asvrl_iqn_train_fused(C.byref(pack.struct), C.byref(pack.head), C.byref(io),
                                                C.byref(parts), _abi.stream_ptr(stream)), "asvrl_iqn_train_fused",
                   pack.L)
    for (layer, M, K), part in zip(shapes, regions):
        arena.groups(part, groups, M, K, layer.weight.grad, layer.bias.grad)
    if encoders:
        arena._seg(enc_part, gs[0], None, groups, 688, 0, False)


def iqn_act(pack, F, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed, taus=None,
            stream=None, obs=None):
    """act_iqn for every row of F (or of the observation rows `obs`) into actions64[:, 0] (f64 action index)."""
    io = _io(F, K_ACT, obs=obs, taus=taus, act_out=actions64, ld_act=actions64.stride(0), step_dev=step_dev,
             eps_steps_per_count=float(steps_per_count), eps_total=float(total), eps_fraction=float(fraction),
             eps_initial=float(initial), eps_final=float(final), seed=int(seed) & 0xFFFFFFFFFFFFFFFF)
    _abi.check(pack.L.asvrl_iqn_act(C.byref(pack.struct), C.byref(pack.head), C.byref(io),
                                    _abi.stream_ptr(stream)), "asvrl_iqn_act", pack.L)


class FusedIQNState:
    """Packs and buffers of the fused IQN update (allocated once, pointer-stable for graphs).
    operands="f32": every kernel from libasvrl_f32.so (the parity build; the optimiser must be a
    FusedAdam of the same operands)."""

    def __init__(self, net_local, net_target, B, N, operands="bf16", target_in_fused=None):
        dev = net_local.cos_embedding.weight.device
        self.B, self.N, self.device = B, N, dev
        self.operands = operands
        # the target's max inside the fused launch (bf16 build; module default TARGET_IN_FUSED)
        self.target_in_fused = TARGET_IN_FUSED if target_in_fused is None else bool(target_in_fused)
        self.A = net_local.action_size
        self.local = IqnPack(net_local, operands)
        self.target = IqnPack(net_target, operands)
        self.bufs = TrainBuffers(B, N, dev, operands)
        f = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=_abi.operand_dtype(operands), device=dev)
        self.xb = torch.empty(B, 32, **bf)
        self.q_next = torch.empty(B * N, **f)
        self.dzF = torch.empty(B, 256, **bf)
        self.dz_out = torch.empty(B * N, _abi.IQN_MAX_ACTIONS, **bf)
        self.arena = PartialArena(32 << 20, dev, operands)
        self.loss = torch.zeros(1, **f)
        self.tile_loss = torch.zeros(B * N // 32, **f)

    def target_changed(self):
        """Re-pack the target network after a hard/soft update (eager, outside graphs)."""
        self.target.refresh()

    def act(self, obs_rows, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed):
        iqn_act(self.local, None, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed,
                obs=obs_rows)


def iqn_grads(st, net, rows, taus, gamma=0.99, flush=True):
    """train_IQN's backward (agent.py:449-468) for replay rows [B][88] and taus (2, B, N) =
    (target, local): every parameter .grad and st.loss. flush=False leaves the weight-gradient
    partials queued on st.arena (the update reduces them together with the gradient norm)."""
    B, N = st.B, st.N
    s_rows, ns_rows = rows[:, 0:OBS], rows[:, OBS:2 * OBS]
    a_col, r_col, d_col = rows[:, 80], rows[:, 82], rows[:, 83]
    bufs, arena = st.bufs, st.arena
    # every .grad is overwritten below (no zeroing); the trunk kernels run the encoders on the rows
    fused = FUSED_TRAIN and fused_train_supported(st.local, B, N)
    target_in = fused and ENC_IN_KERNEL and st.target_in_fused and st.operands == "bf16"
    if not target_in:
        iqn_forward_max(st.target, None, taus[0], N, st.q_next, obs=ns_rows)
    if fused:
        # forward, loss, backward and the four layers' weight-gradient partials in one launch
        if ENC_IN_KERNEL:   # ... and the encoders' gradient partials (and, target_in, the target's max first)
            iqn_train_fused(st.local, net, taus[1], N, st.q_next.view(B, N), a_col, r_col, d_col, gamma, s_rows,
                            arena, tile_loss=st.tile_loss, encoders=True,
                            target=(st.target, taus[0], ns_rows) if target_in else None)
        else:
            iqn_train_fused(st.local, net, taus[1], N, st.q_next.view(B, N), a_col, r_col, d_col, gamma, s_rows,
                            arena, dzF=st.dzF, xb=st.xb, tile_loss=st.tile_loss)
            with arena.batch():
                arena.fold(st.dzF, st.xb, net)   # encoder image -> self/object encoder grads
        arena.scalar(st.tile_loss, st.loss)
        if flush:
            arena.flush()
        return
    iqn_train(st.local, None, taus[1], bufs, st.dz_out, st.q_next.view(B, N), a_col, r_col, d_col, gamma, st.dzF,
              tile_loss=st.tile_loss, obs=s_rows, xb=st.xb)
    with arena.batch():   # the five layers in one launch
        # the padded 32-row output reduction fills the A-row output layer directly
        arena.linear(st.dz_out, bufs.h2, net.output_layer.weight.grad, net.output_layer.bias.grad)
        arena.linear(bufs.dzc, bufs.cos, net.cos_embedding.weight.grad, net.cos_embedding.bias.grad)
        arena.fold(st.dzF, st.xb, net)   # encoder image -> self/object encoder grads
        arena.linear(bufs.dz1, bufs.h0, net.hidden_layer.weight.grad, net.hidden_layer.bias.grad)
        arena.linear(bufs.dz2, bufs.h1g, net.hidden_layer_2.weight.grad, net.hidden_layer_2.bias.grad)
    arena.scalar(st.tile_loss, st.loss)
    if flush:
        arena.flush()


def iqn_update_fused(st, net, opt, grads, rows, gamma=0.99, taus=None, sync=None, max_norm=0.5, act_wait=None,
                     counter=None):
    """One IQN update from replay rows [B][88]; taus: (2, B, N) (target, local) or None (drawn).
    act_wait: event to wait for before the weights change (a concurrent act kernel).
    Returns (loss, grad_norm) as device scalars."""
    if taus is None:
        taus = torch.rand(2, st.B, st.N, device=st.device)
    iqn_grads(st, net, rows, taus, gamma, flush=False)
    gn = _reduce_and_step(st.arena, opt, grads, sync, max_norm, wait=act_wait, pack=st.local, counter=counter)
    return st.loss[0], gn
