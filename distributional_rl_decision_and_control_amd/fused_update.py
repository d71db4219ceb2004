"""The whole AC-IQN update (Agent.train_AC_IQN, agent.py:386-432) on hand-written gfx950
kernels: eight launches per step (with the vectorised loop's fused prologue and the target critic inside the
critic launch), no torch autograd, no host synchronisation.

Per step, on a replay batch `rows` ([B][88]: obs | next obs | action | reward | done):
  actor(s) saving activations -> a (for the actor step)  asvrl_actor_forward(TRAIN)
  critic (agent.py:395-416)
    target actor(ns) -> na                               asvrl_actor_forward(FWD)
    target encoders(ns, na) + trunk -> q_next            asvrl_critic_forward (encoders in the prologue);
                                                          (by default inside the next launch: TARGET_IN_FUSED,
                                                          ABI 20, asvrl_critic_train_fused_tq)
    local encoders(s, a), trunk forward, quantile-Huber vs r + g q_next (1-d), backward AND the
    four trunk layers' weight-gradient partials          asvrl_critic_train_fused (ONE launch)
    and the observation / action encoders' gradient partials (ABI 16; ENC_IN_KERNEL = False: from
    dzF / dzG by ONE asvrl_linear_wgrad_multi, fold + small)
    every .grad (encoders folded in the reduction), the loss and the global gradient norm
                                                          ONE asvrl_partial_sums_norm
    clip + Adam + re-pack of the weight images           asvrl_adam_step_pack
      (with DP: asvrl_partial_sums, RCCL all-reduce, asvrl_partial_sums_norm over the averaged gradient
       (FusedAdam.step_synced), asvrl_adam_step_pack)
  actor (agent.py:419-427), through the UPDATED critic
    encoders(s, a) + trunk forward + backward of -mean(q) to the action
                                                          asvrl_critic_actor_grad (dA in-kernel)
    actor backward                                       asvrl_actor_backward
    every actor .grad, the actor loss, the norm partials  ONE asvrl_actor_grads (split tiles reduced in-launch)
    clip + Adam + re-pack                                asvrl_adam_step_pack
(supported() admits only shapes the fused critic launch takes: B a multiple of 32, so B*N one of its
64-row round.)

The learner runs on the caller's stream (a replayed graph pays ~10 us per cross-stream join; the only
other stream is the rollout's, vec_trainer.py).

Arithmetic: bf16 MFMA operands with f32 accumulation everywhere, f32 master weights / Adam
(operands="f32": the same kernels from libasvrl_f32.so, the parity build).
"""
import ctypes as C

import torch

from . import _abi
from .fused_critic import CriticPack, PartialArena, critic_actor_grad, critic_forward, critic_train_fused
from .fused_mlp import (ActorBuffers, ActorGrads, MlpPack, actor_act, actor_backward, actor_forward,
                        actor_train_forward)
from .fused_mlp import actor_grads as actor_grads_launch
from .learner import FusedAdam, clip_and_step

OBS = 40
# the encoders' gradients formed inside the fused critic launch (ABI 16: 0.333 -> 0.323 ms per AC-IQN
# step, profiles/r02_enc_ab.txt); False keeps the earlier form (per-sample dzF / dzG + a batched launch)
# for the kernel tests that compare the two
ENC_IN_KERNEL = True
# the target critic's forward inside the fused critic launch (ABI 20, asvrl_critic_train_fused_tq: each
# workgroup computes q_next for the samples it updates, bit-identical to the separate asvrl_critic_forward).
# Round 4 measured it slower (0.2649 vs 0.2629 ms, profiles/r04t_target_in_fused_ab.txt); at the round-5 head
# (leaner epilogues, the one-launch auto-reset) the separate target launch costs 54 us beside the next env step
# while the in-launch pass adds ~35 us to the update, and the step is faster: 0.2591 vs 0.2642 ms at the
# driver's shape, 0.2478 vs 0.2503 at steady state (profiles/r05ac_target_in_fused_ab.txt)
TARGET_IN_FUSED = True


def supported(policy, B, N):
    c, a = policy.critic, policy.actor
    return (c.concat_feature_dimension == 256 and c.hidden_dimension == 128 and c.n == 64 and N in (8, 16, 32)
            and (B * N) % 32 == 0 and B % 32 == 0 and c.self_dimension == 7 and c.object_dimension == 5
            and c.max_object_num == 5 and c.self_feature_dimension == 56 and c.object_feature_dimension == 40
            and a.hidden_dimension == 128 and a.concat_feature_dimension == 256 and a.action_dimension == 2
            and c.action_dimension == 2)


class FusedACIQNState:
    """Packs and buffers of the fused update (allocated once, pointer-stable for graph replay).
    operands="f32": every kernel from libasvrl_f32.so, the f32-operand parity build of the same
    sources (the optimisers must be FusedAdam of the same operands)."""

    def __init__(self, policy_local, policy_target, B, N, operands="bf16", double_actor=False):
        dev = policy_local.critic.cos_embedding.weight.device
        self.B, self.N, self.device = B, N, dev
        self.operands = operands
        # the critic's encoders run inside the trunk kernels (f32, straight from the parameters)
        self.local_trunk = CriticPack(policy_local.critic, operands)
        self.target_trunk = CriticPack(policy_target.critic, operands)
        # double_actor (the batched loop): two actor image sets, the optimiser writing the one the act kernel
        # does not read (MlpPack)
        self.actor = MlpPack(policy_local.actor, "actor", operands, double=double_actor)
        self.target_actor = MlpPack(policy_target.actor, "actor", operands)
        self.abufs = ActorBuffers(B, dev, operands)
        self.agrads = ActorGrads(B, dev, operands)
        f = dict(dtype=torch.float32, device=dev)
        bf = dict(dtype=_abi.operand_dtype(operands), device=dev)
        self.na = torch.empty(B, 2, **f)
        self.xb = torch.empty(B, 32, **bf)
        self.q_next = torch.empty(B * N, **f)
        self.q_pi = torch.empty(B * N, **f)
        self.dzF = torch.empty(B, 256, **bf)
        self.dzG = torch.empty(B, 128, **f)
        self.arena = PartialArena(32 << 20, dev, operands)
        self.losses = torch.zeros(2, **f)   # critic, actor loss (summed from per-tile partials)
        self.tile_loss = torch.zeros(2, B * N // 32, **f)

    def target_changed(self):
        """Re-pack the target networks after a hard/soft update (eager, outside graphs)."""
        self.target_trunk.refresh()
        self.target_actor.refresh()

    def act(self, obs_rows, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed):
        actor_act(self.actor, obs_rows, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed)


def _reduce_and_step(arena, opt, grads, sync, max_norm, wait=None, pack=None, counter=None):
    """Reduce the queued weight-gradient partials, then clip + Adam. Single process with the
    fused optimiser: the reduction launch also forms the gradient norm and the Adam launch writes the
    weight images of `pack` (a CriticPack / MlpPack / IqnPack) and increments `counter` (two launches
    in all; one persistent launch with a grid barrier between the two was measured slower);
    with FusedAdam and a data-parallel `sync`: reduce (asvrl_partial_sums), all-reduce, then FusedAdam.step_synced
    (asvrl_partial_sums_norm over the averaged gradient + the same packing asvrl_adam_step_pack); with another
    optimiser: reduce, all-reduce, clip_and_step, then pack.refresh() and counter += 1.
    `wait`: an event to wait for before the parameters change."""
    assert pack is None or not isinstance(opt, FusedAdam) or opt.L is pack.L, "optimiser and pack of different builds"
    if isinstance(opt, FusedAdam):
        # the fused steps clip at the optimiser's own max_norm: refuse a different one rather than ignore it
        assert opt.max_norm == max_norm, (opt.max_norm, max_norm)
        if pack is not None and not hasattr(pack, "_adam_segs"):
            pack._adam_segs = pack.adam_segments(opt)
        segs = pack._adam_segs if pack is not None else None
        if sync is None:
            arena.flush(norm=opt)
            if wait is not None:
                torch.cuda.current_stream().wait_event(wait)
            return opt.step_prenormed(arena.norm_parts, arena.nparts, pack=segs, counter=counter)
        # data-parallel: reduce, all-reduce, then the norm over the averaged gradient and the same packing
        # Adam launch (no re-pack launches, no counter op: DP step 0.316 ms with them)
        arena.flush()
        sync(grads)
        if wait is not None:
            torch.cuda.current_stream().wait_event(wait)
        return opt.step_synced(pack=segs, counter=counter)
    gn = _step_unfused(arena, opt, grads, sync, max_norm, wait)
    if pack is not None:
        pack.refresh()
    if counter is not None:
        counter += 1
    return gn


def _step_unfused(arena, opt, grads, sync, max_norm, wait):
    arena.flush()
    if sync is not None:
        sync(grads)
    if wait is not None:
        torch.cuda.current_stream().wait_event(wait)
    return clip_and_step(opt, grads, max_norm)


def target_q(st, rows, tau0, q_out, na):
    """Q_targets_next of agent.py:397-400 for the rows' next states: target actor, then the target
    critic with the target encoders inside the trunk kernel (q_out [B*N])."""
    ns_rows = rows[:, OBS:2 * OBS]
    actor_forward(st.target_actor, ns_rows, na)
    critic_forward(st.target_trunk, None, None, tau0, st.N, q=q_out, obs=ns_rows, act=na)


def learn_prologue(st, replay, taus, seed, counter_dev=None, counter=0, out=None, state=None, guard=0, stream=None):
    """asvrl_learn_prologue: B rows drawn from the device ring (replay_buffer.py:26-45) with the update's
    quantile fractions `taus` (3, B, N), the local actor's TRAIN forward on s (its activations in st.abufs)
    and the target actor's forward on s' (st.na) in ONE launch, bit-identical to replay.sample +
    actor_train_forward + actor_forward. Returns the rows [B][88]."""
    B = st.B
    out = out if out is not None else torch.empty((B, 88), dtype=torch.float32, device=st.device)
    assert taus.is_contiguous() and taus.shape[1] == B and taus.dtype == torch.float32
    sa = _abi.AsvSampleArgs()
    sa.ring, sa.capacity = replay.ring.data_ptr(), replay.capacity
    sa.ring_state = (state if state is not None else replay.state).data_ptr()
    sa.seed, sa.counter = int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF
    sa.counter_dev = _abi.ptr(counter_dev)
    sa.guard, sa.B, sa.tau_sets, sa.tau_n = int(guard), B, taus.shape[0], taus.shape[2]
    sa.out, sa.taus = out.data_ptr(), taus.data_ptr()
    io = st.abufs.io()
    _abi.check(st.actor.L.asvrl_learn_prologue(C.byref(sa), C.byref(st.actor.w), C.byref(io),
                                                C.byref(st.target_actor.w), st.na.data_ptr(),
                                                _abi.stream_ptr(stream)), "asvrl_learn_prologue", st.actor.L)
    return out


def ac_iqn_update_fused2(st, policy_local, actor_opt, critic_opt, critic_grads, actor_grads, rows, gamma=0.99,
                         taus=None, sync=None, max_norm=0.5, actor_wait=None, counter=None, prologue_done=False,
                         target_wait=None, actor_done=None):
    """One AC-IQN update from replay rows [B][88]. taus: (3, B, N) or None (drawn here).
    actor_wait: event to wait for before the actor's weights change (a concurrent act kernel).
    counter: an int64 device scalar incremented after the step (the learn counter; in-kernel when
    the optimiser step is fused). prologue_done: learn_prologue already ran the actor's TRAIN forward and
    the target actor on these rows. target_wait: an event the target critic waits for (a schedule knob:
    the rollout's env step ahead of it instead of beside it; no data dependency) -- with the target pass inside the
    fused launch (TARGET_IN_FUSED) the whole fused critic update waits for it. actor_done: an event recorded
    after the ACTOR pass (a schedule knob: what the rollout's replay push may wait for).
    Returns (critic_loss, actor_loss, critic_grad_norm, actor_grad_norm) as device scalars."""
    B, N = st.B, st.N
    critic, actor = policy_local.critic, policy_local.actor
    if taus is None:
        taus = torch.rand(3, B, N, device=st.device)
    s_rows = rows[:, 0:OBS]
    a_rows, r_col, d_col = rows[:, 80:82], rows[:, 82], rows[:, 83]
    ab, arena = st.abufs, st.arena

    # ---- critic (agent.py:395-416); every critic .grad is overwritten below (no zeroing). The
    # trunk kernels run the critic's observation / action encoders on the replay rows themselves.
    q_next = st.q_next
    if target_wait is not None:
        torch.cuda.current_stream().wait_event(target_wait)
    # the target critic's forward inside the update's launch (each workgroup for its own samples): one
    # launch fewer on the learner chain
    target_in = TARGET_IN_FUSED and prologue_done and ENC_IN_KERNEL
    if target_in:
        pass
    elif prologue_done:   # only the target critic is left of the target chain
        critic_forward(st.target_trunk, None, None, taus[0], st.N, q=q_next, obs=rows[:, OBS:2 * OBS], act=st.na)
    else:
        actor_train_forward(st.actor, s_rows, ab)   # reads only s and the (not yet updated) actor
        target_q(st, rows, taus[0], q_next, st.na)
    ae = critic.action_encoder[0]
    # forward, loss, backward and the weight-gradient partials of the four trunk layers and the three
    # encoders in one launch (supported() guarantees its shape: B a multiple of 32, so B*N of 64)
    if ENC_IN_KERNEL:
        critic_train_fused(st.local_trunk, critic, taus[1], N, q_next.view(B, N), r_col, d_col, gamma, s_rows,
                           a_rows, arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=(st.target_trunk, taus[0], rows[:, OBS:2 * OBS], st.na) if target_in else None)
    else:
        critic_train_fused(st.local_trunk, critic, taus[1], N, q_next.view(B, N), r_col, d_col, gamma, s_rows,
                           a_rows, arena, dzF=st.dzF, dzG=st.dzG, xb=st.xb, tile_loss=st.tile_loss[0])
        with arena.batch():   # the encoders' gradients from the per-sample dzF / dzG
            arena.fold(st.dzF, st.xb, critic)
            arena.small(st.dzG, a_rows, ae.weight.grad, ae.bias.grad)
    arena.scalar(st.tile_loss[0], st.losses[0:1])   # the critic loss
    cgn = _reduce_and_step(arena, critic_opt, critic_grads, sync, max_norm, pack=st.local_trunk)

    # ---- actor through the updated critic (agent.py:419-427)
    critic_actor_grad(st.local_trunk, None, None, taus[2], N, st.q_pi, w_ae=ae.weight, dA=ab.dA,
                      tile_loss=st.tile_loss[1], obs=s_rows, act=ab.a_out)
    if actor_done is not None:   # behind the ACTOR pass (behind the actor's backward measured no better, r05aq)
        actor_done.record(torch.cuda.current_stream())
    actor_backward(st.actor, ab)
    # every actor .grad, the actor loss, the norm partials and the Adam step count in one launch
    fused_opt = sync is None and isinstance(actor_opt, FusedAdam)
    actor_grads_launch(st.agrads, ab, actor, st.tile_loss[1], st.losses[1:2],
                       step=actor_opt.step_t if fused_opt else None, norm=fused_opt)
    if isinstance(actor_opt, FusedAdam):
        assert actor_opt.max_norm == max_norm, (actor_opt.max_norm, max_norm)
        if sync is not None:
            sync(actor_grads)
        # a concurrent act kernel reads the current actor images: with two sets the step writes the other one
        # and no wait is needed (its cross-stream dependency costs ~7 us in a replayed graph)
        if actor_wait is not None and not st.actor.double:
            torch.cuda.current_stream().wait_event(actor_wait)
        if fused_opt:
            agn = actor_opt.step_prenormed(st.agrads.norm_parts, st.agrads.nparts,
                                           pack=st.actor.adam_segments(actor_opt), counter=counter)
        else:   # data-parallel: the norm over the all-reduced gradient, then the same packing step
            agn = actor_opt.step_synced(pack=st.actor.adam_segments(actor_opt), counter=counter)
        st.actor.flip()
    else:
        if sync is not None:
            sync(actor_grads)
        if actor_wait is not None:
            torch.cuda.current_stream().wait_event(actor_wait)
        agn = clip_and_step(actor_opt, actor_grads, max_norm)
        st.actor.refresh()
        if counter is not None:
            counter += 1
    return st.losses[0], st.losses[1], cgn, agn
