"""Optimiser and data-parallel plumbing of the learner (agent.py:75-76, 98, 415-427), and the
torch-autograd update functions the drop-in Agent falls back to for network shapes the kernels do not take.

* FlatGrads / FusedAdam: every network's gradient in one flat buffer; clip + Adam (+ the re-pack of the
  kernels' bf16 weight images) as hand-written launches (asvrl_adam_clip, asvrl_adam_step_pack).
* GradSync: the data-parallel all-reduce of a flat gradient over RCCL between the gradient reduction and the
  clip -- twice per AC-IQN step (critic, then actor through the *updated* critic, agent.py:395-427), once for
  IQN / Rainbow.
* ac_iqn_update / iqn_update / rainbow_update: the reference's updates on torch modules (autograd) with the
  quantile-Huber loss (learn_ops.quantile_huber_loss) and the C51 projection (learn_ops.c51_project) on their
  kernels. The training path does not use them: its updates are the fused launches of fused_update.py,
  fused_iqn.py and fused_rainbow.py (no torch GEMM, no autograd); Agent uses these only for shapes those
  launches do not take, and says so when it does (agent.py).
"""
import ctypes as C

import torch
import torch.distributed as dist

from . import _abi
from ._abi import OBS_DIM
from .learn_ops import c51_project, quantile_huber_loss


class FlatGrads:
    """Gives every parameter of `params` a .grad that is a view into one flat buffer, so a
    gradient all-reduce is one collective on contiguous memory."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero_(self):
        self.flat.zero_()

    def assign(self, grads):
        torch._foreach_copy_([p.grad for p in self.params], list(grads))


class GradSync:
    """All-reduce(average) of a FlatGrads buffer over the default process group (RCCL on
    MI355X: backend "nccl"; gloo on CPU tests)."""

    def __init__(self, group=None, force=False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.avg_supported = dist.is_initialized() and dist.get_backend(group) == "nccl"
        # force: issue the collective even over one rank (tests of the captured DP path on one GPU)
        self.force = bool(force) and dist.is_initialized()
        # timing: None, or a list that collects (bytes, start event, end event) per collective -- HIP events on
        # the stream the collective is issued on (RCCL runs on it), eager steps only (bench.py allreduce_timing)
        self.timing = None

    def __call__(self, fg: FlatGrads):
        if self.world == 1 and not self.force:
            return
        if self.timing is not None and fg.flat.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream(fg.flat.device))
            self._reduce(fg)
            e1.record(torch.cuda.current_stream(fg.flat.device))
            self.timing.append((fg.flat.numel() * fg.flat.element_size(), e0, e1))
            return
        self._reduce(fg)

    def _reduce(self, fg):
        if self.avg_supported:
            dist.all_reduce(fg.flat, op=dist.ReduceOp.AVG, group=self.group)
        elif fg.flat.is_cuda:
            # gloo (CPU-side tests of the multi-rank GPU path): stage through host memory
            host = fg.flat.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            fg.flat.copy_(host.div_(self.world))
        else:
            dist.all_reduce(fg.flat, op=dist.ReduceOp.SUM, group=self.group)
            fg.flat.div_(self.world)


def _clip(params, max_norm):
    return torch.nn.utils.clip_grad_norm_(params, max_norm)


class FusedAdam:
    """clip_grad_norm_(params, max_norm) + optim.Adam(params, lr).step() (agent.py:75-76,98,
    415-416) as the two launches of asvrl_adam_clip over flat buffers.

    The parameters are re-pointed at one flat f32 buffer (p.data becomes a view, so modules,
    state_dict and load_state_dict keep working) and their .grad at a FlatGrads buffer in the
    same order; `grads` is that FlatGrads, to be all-reduced by GradSync before step().
    Construct it before anything caches parameter pointers (CriticPack)."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, max_norm=0.5, operands="bf16"):
        # operands: the learner build whose weight images asvrl_adam_step_pack writes (bf16 / f32)
        self.L = _abi.lib(operands)
        self.params = [p for p in params if p.requires_grad]
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.flat[off:off + k].copy_(p.reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                off += k
        self.grads = FlatGrads(self.params)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.work = torch.zeros(64, dtype=torch.float64, device=dev)
        self.lr, self.betas, self.eps, self.max_norm = float(lr), tuple(betas), float(eps), float(max_norm)
        self.n = n

    def zero_grad(self):
        self.grads.zero_()

    def step(self):
        """Clip + Adam; returns the pre-clip global norm as a 0-d device tensor."""
        rc = self.L.asvrl_adam_clip(
            _abi.ptr(self.flat), _abi.ptr(self.grads.flat), _abi.ptr(self.exp_avg), _abi.ptr(self.exp_avg_sq),
            self.n, _abi.ptr(self.step_t), self.lr, self.betas[0], self.betas[1], self.eps, self.max_norm,
            _abi.ptr(self.norm), _abi.ptr(self.work), _abi.stream_ptr(None))
        _abi.check(rc, "asvrl_adam_clip", self.L)
        return self.norm[0]

    def pack_seg(self, w, image, K=0, chained=False, transposed=False, f32=False, row0=0, col0=0, nrep=1, rep_row=0,
                 rep_col=0):
        """An AsvPackSeg sending parameter w (one of this optimiser's, re-pointed into its flat buffer)
        into a weight image at every step (asvrl_adam_step_pack)."""
        off = (w.data_ptr() - self.flat.data_ptr()) // 4
        assert 0 <= off and off + w.numel() <= self.n and w.is_contiguous()
        g = _abi.AsvPackSeg()
        g.flat_off, g.image = off, image.data_ptr()
        g.rows, g.cols = (w.shape[0], w.shape[1]) if w.dim() == 2 else (w.shape[0], 1)
        g.K, g.chained, g.transposed, g.f32 = K, int(chained), int(transposed), int(f32)
        g.row0, g.col0, g.nrep, g.rep_row, g.rep_col = row0, col0, nrep, rep_row, rep_col
        return g

    def step_synced(self, pack=None, counter=None, stream=None):
        """Clip + Adam over gradients already reduced in place (the data-parallel path, after GradSync's
        all-reduce): one asvrl_partial_sums_norm launch over the flat gradient as a single one-group segment
        (it rewrites each value in place, leaves the squared-norm partials and advances step_t), then the
        step_prenormed launch, which writes the weight images of `pack` and increments `counter` -- instead
        of asvrl_adam_clip followed by a re-pack of every image and a counter op. Returns the pre-clip norm."""
        if getattr(self, "_sync_seg", None) is None:
            g = _abi.AsvPartialSum()
            g.partial = g.dw = self.grads.flat.data_ptr()
            g.db = None
            g.groups, g.nw, g.nb, g.accumulate = 1, self.n, 0, 0
            g.stride, g.boff, g.mode, g.norm = 0, 0, _abi.SUM_PLAIN, 1
            self._sync_seg = (_abi.AsvPartialSum * 1)(g)
            self._sync_nparts = int(self.L.asvrl_partial_sums_norm_parts(self._sync_seg, 1))
            self._sync_parts = torch.zeros(self._sync_nparts, dtype=torch.float64, device=self.flat.device)
        _abi.check(self.L.asvrl_partial_sums_norm(self._sync_seg, 1, _abi.ptr(self._sync_parts), _abi.ptr(self.step_t),
                                                  _abi.stream_ptr(stream)), "asvrl_partial_sums_norm", self.L)
        return self.step_prenormed(self._sync_parts, self._sync_nparts, pack=pack if pack is not None else [],
                                   counter=counter)

    def step_prenormed(self, norm_parts, nparts, pack=None, counter=None):
        """Clip + Adam with the squared norm as nparts f64 partials and step_t already advanced
        (PartialArena.flush(norm=self)): one launch. pack: AsvPackSeg list -- the same launch writes
        the updated weights into those images (no re-pack launch); counter: an int64 device scalar
        the launch increments. Returns the pre-clip norm."""
        if pack or counter is not None:
            pack = list(pack or [])
            arr = (_abi.AsvPackSeg * max(1, len(pack)))(*pack)
            rc = self.L.asvrl_adam_step_pack(
                _abi.ptr(self.flat), _abi.ptr(self.grads.flat), _abi.ptr(self.exp_avg), _abi.ptr(self.exp_avg_sq),
                self.n, _abi.ptr(self.step_t), self.lr, self.betas[0], self.betas[1], self.eps, self.max_norm,
                _abi.ptr(self.norm), _abi.ptr(norm_parts), int(nparts), arr, len(pack),
                _abi.ptr(counter) if counter is not None else None, _abi.stream_ptr(None))
            _abi.check(rc, "asvrl_adam_step_pack", self.L)
            return self.norm[0]
        rc = self.L.asvrl_adam_step(
            _abi.ptr(self.flat), _abi.ptr(self.grads.flat), _abi.ptr(self.exp_avg), _abi.ptr(self.exp_avg_sq),
            self.n, _abi.ptr(self.step_t), self.lr, self.betas[0], self.betas[1], self.eps, self.max_norm,
            _abi.ptr(self.norm), _abi.ptr(norm_parts), int(nparts), _abi.stream_ptr(None))
        _abi.check(rc, "asvrl_adam_step", self.L)
        return self.norm[0]


def clip_and_step(opt, grads, max_norm):
    """Global-norm clip then optimizer step; returns the pre-clip norm (device scalar)."""
    if isinstance(opt, FusedAdam):
        assert opt.max_norm == max_norm and opt.grads.flat.data_ptr() == grads.flat.data_ptr()
        return opt.step()
    n = _clip(grads.params, max_norm)
    opt.step()
    return n


def ac_iqn_update(policy_local, policy_target, actor_opt, critic_opt, critic_grads, actor_grads, states, actions,
                  rewards, next_states, dones, gamma=0.99, num_tau=8, taus=(None, None, None), sync=None,
                  amp_dtype=None, max_norm=0.5):
    """train_AC_IQN (agent.py:386-432). rewards/dones (B, 1). Returns (critic_loss, actor_loss,
    critic_grad_norm, actor_grad_norm) as 0-d device tensors (no host sync)."""
    actor, critic = policy_local.actor, policy_local.critic
    amp = torch.autocast("cuda", dtype=amp_dtype) if amp_dtype is not None else _null()
    # ---- critic (agent.py:395-416)
    critic_grads.zero_()
    with torch.no_grad(), amp:
        next_actions = policy_target.actor(next_states)
        q_next, _ = policy_target.critic(next_states, next_actions, num_tau, taus=taus[0])
    q_next = q_next.float()
    q_targets = rewards + gamma * q_next * (1.0 - dones)  # (B, N')
    with amp:
        q_exp, tau_e = critic(states, actions, num_tau, taus=taus[1])
    critic_loss = quantile_huber_loss(q_targets, q_exp.float(), tau_e)
    critic_loss.backward()
    if sync is not None:
        sync(critic_grads)
    cgn = clip_and_step(critic_opt, critic_grads, max_norm)
    # ---- actor through the updated critic (agent.py:419-427); only actor grads are needed
    with amp:
        a_out = actor(states)
        q_pi, _ = critic(states, a_out, num_tau, taus=taus[2])
    actor_loss = -q_pi.float().mean()
    g = torch.autograd.grad(actor_loss, actor_grads.params)
    actor_grads.assign(g)
    if sync is not None:
        sync(actor_grads)
    agn = clip_and_step(actor_opt, actor_grads, max_norm)
    return critic_loss.detach(), actor_loss.detach(), cgn, agn


def iqn_update(policy_local, policy_target, opt, grads, states, actions, rewards, next_states, dones, gamma=0.99,
               num_tau=8, taus=(None, None), sync=None, amp_dtype=None, max_norm=0.5):
    """train_IQN (agent.py:434-476); actions (B,) int64. Target = max over actions per tau
    sample (agent.py:452), not argmax of the mean."""
    amp = torch.autocast("cuda", dtype=amp_dtype) if amp_dtype is not None else _null()
    grads.zero_()
    with torch.no_grad(), amp:
        qn, _ = policy_target(next_states, num_tau, taus=taus[0])
    qn = qn.float().max(2)[0]  # (B, N)
    q_targets = rewards + gamma * qn * (1.0 - dones)
    with amp:
        qe, tau_e = policy_local(states, num_tau, taus=taus[1])
    B = qe.shape[0]
    qe = qe.float().gather(2, actions.view(B, 1, 1).expand(B, num_tau, 1)).squeeze(-1)
    loss = quantile_huber_loss(q_targets, qe, tau_e)
    loss.backward()
    if sync is not None:
        sync(grads)
    gn = clip_and_step(opt, grads, max_norm)
    return loss.detach(), gn


def rainbow_update(policy_local, policy_target, opt, grads, support, states, actions, returns, next_states,
                   nonterminals, weights, gamma=0.99, n=3, vmin=-1.0, vmax=1.0, sync=None, max_norm=0.5,
                   reset_target_noise=True):
    """train_Rainbow (agent.py:597-641) with the projection on the C51 kernel. Returns the
    per-sample loss (for update_priorities) and the pre-clip grad norm."""
    B = actions.shape[0]
    log_ps = policy_local(states, log=True)
    log_ps_a = log_ps[torch.arange(B, device=actions.device), actions]
    with torch.no_grad():
        pns = policy_local(next_states)
        dns = support.expand_as(pns) * pns
        argmax_ns = dns.sum(2).argmax(1)
        if reset_target_noise:
            policy_target.reset_noise()
        pns = policy_target(next_states)
        pns_a = pns[torch.arange(B, device=actions.device), argmax_ns]
        m = c51_project(pns_a, returns, nonterminals, support, vmin, vmax, gamma ** n)
    loss = -torch.sum(m * log_ps_a, 1)
    grads.zero_()
    (weights * loss).mean().backward()
    if sync is not None:
        sync(grads)
    gn = clip_and_step(opt, grads, max_norm)
    return loss.detach(), gn


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
