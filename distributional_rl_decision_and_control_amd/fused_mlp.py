"""Per-row MLPs of AC-IQN on the gfx950 kernels of csrc/asvrl_mlp.hip.

MlpPack holds the bf16 images one network's per-row layers are read from (both observation
encoders as a single block-structured 256 x 32 matrix, the Actor's hidden layers in the chained
fragment order plus their transposes, the critic's action encoder) and refreshes them in one
launch (asvrl_mlp_pack) after every optimizer step. The wrappers below are thin: tensors in,
device pointers out, no host synchronisation, so everything is capturable in a HIP graph.

Reference layers: AC_IQN_model.py:254-262 (Actor), 389-404 (Critic encoders), forward passes
:284-321 and :462-480.
"""
import ctypes as C

import torch

from . import _abi

ENC, OBSK, HID = 256, 32, 128
MAX_OBJ = 5   # object-encoder copies in the encoder image (max_object_num)
MODE_ACT, MODE_FWD, MODE_TRAIN = 1, 2, 3


def _p(t):
    return t.data_ptr() if t is not None else None


class MlpPack:
    """Packed images of an Actor (kind='actor'), of a Critic's encoders + action encoder
    (kind='critic') or of the observation encoders alone (kind='encoders', IQN_Policy).
    operands="f32": f32 images for libasvrl_f32.so (the parity build); launches go to self.L.

    double=True (an Actor in the batched loop): two image sets, with f32 copies of the biases and the output
    layer in each. Launches read set `parity` (self.w); the optimiser step writes the other one
    (adam_segments) and flip() makes it current -- so the rollout's act kernel, which reads the current set,
    never races the step that rewrites the weights (no cross-stream wait before the optimiser)."""

    def __init__(self, net, kind, operands="bf16", double=False):
        assert kind in ("actor", "critic", "encoders")
        assert not double or kind == "actor"
        self.net, self.kind = net, kind
        self.operands = operands
        self.L = _abi.lib(operands)
        self.double = double
        self.parity = 0
        self.sets = [self._make_set(net, kind, operands, double) for _ in range(2 if double else 1)]
        self._segs = {}
        self.refresh()

    @staticmethod
    def _make_set(net, kind, operands, copies):
        dev = net.self_encoder[0].weight.device
        bf = dict(dtype=_abi.operand_dtype(operands), device=dev)
        f = dict(dtype=torch.float32, device=dev)
        t = {"enc": torch.zeros(ENC * OBSK, **bf), "b_enc": torch.zeros(ENC, **f)}
        w = _abi.AsvMlpWeights()
        w.enc_frag, w.b_enc = t["enc"].data_ptr(), t["b_enc"].data_ptr()
        if kind == "actor":
            for k, n in (("w1", HID * ENC), ("w2", HID * HID), ("w2t", HID * HID), ("w1t", ENC * HID)):
                t[k] = torch.zeros(n, **bf)
            w.w1_frag, w.w2_frag, w.w2t_frag, w.w1t_frag = (t["w1"].data_ptr(), t["w2"].data_ptr(),
                                                           t["w2t"].data_ptr(), t["w1t"].data_ptr())
            if copies:   # the f32 parameters the kernels read, copied per set
                for k, p in (("b1", net.hidden_layer.bias), ("b2", net.hidden_layer_2.bias),
                             ("wout", net.output_layer.weight), ("bout", net.output_layer.bias)):
                    t[k] = torch.zeros(p.numel(), **f)
                w.b1, w.b2, w.wout, w.bout = (t["b1"].data_ptr(), t["b2"].data_ptr(), t["wout"].data_ptr(),
                                              t["bout"].data_ptr())
            else:
                w.b1, w.b2 = net.hidden_layer.bias.data_ptr(), net.hidden_layer_2.bias.data_ptr()
                w.wout, w.bout = net.output_layer.weight.data_ptr(), net.output_layer.bias.data_ptr()
            w.out_scale = float(net.atan_scale.float().item())
        elif kind == "critic":
            t["ae"] = torch.zeros(HID * 16, **bf)
            w.ae_frag = t["ae"].data_ptr()
            w.b_ae = net.action_encoder[0].bias.data_ptr()
        t["w"] = w
        return t

    @property
    def w(self):
        """The AsvMlpWeights of the current image set."""
        return self.sets[self.parity]["w"]

    def __getattr__(self, name):   # the current set's images: enc, b_enc, w1, w2, w2t, w1t, ae
        sets = self.__dict__.get("sets")
        if sets is not None and name in sets[self.__dict__["parity"]]:
            return sets[self.__dict__["parity"]][name]
        raise AttributeError(name)

    def flip(self):
        """The set the last optimiser step wrote becomes current (double packs; host-side, at enqueue)."""
        if self.double:
            self.parity ^= 1

    def src(self):
        n = self.net
        s = _abi.AsvMlpSrc()
        s.self_w, s.self_b = n.self_encoder[0].weight.data_ptr(), n.self_encoder[0].bias.data_ptr()
        s.obj_w, s.obj_b = n.object_encoder[0].weight.data_ptr(), n.object_encoder[0].bias.data_ptr()
        if self.kind == "actor":
            s.w1, s.w2 = n.hidden_layer.weight.data_ptr(), n.hidden_layer_2.weight.data_ptr()
        elif self.kind == "critic":
            s.ae_w = n.action_encoder[0].weight.data_ptr()
        return s

    def adam_segments(self, opt):
        """The actor's images as AsvPackSeg of FusedAdam `opt` (asvrl_adam_step_pack): the block-structured
        encoder image (self encoder once, the object encoder at its five diagonal blocks), the f32 encoder
        bias copy and the four hidden-layer images -- of the set the step writes (double packs: the other
        set, with the f32 copies of the biases and the output layer; call flip() after the step)."""
        assert self.kind == "actor"
        dst = self.parity ^ 1 if self.double else 0
        if dst in self._segs:
            return self._segs[dst]
        n, t = self.net, self.sets[dst]
        se, oe = n.self_encoder[0], n.object_encoder[0]
        nso, nsi = se.weight.shape
        noo, noi = oe.weight.shape
        W1, W2 = n.hidden_layer.weight, n.hidden_layer_2.weight
        segs = [opt.pack_seg(se.weight, t["enc"], K=OBSK),
                opt.pack_seg(oe.weight, t["enc"], K=OBSK, row0=nso, col0=nsi, nrep=MAX_OBJ, rep_row=noo, rep_col=noi),
                opt.pack_seg(se.bias, t["b_enc"], f32=True),
                opt.pack_seg(oe.bias, t["b_enc"], f32=True, row0=nso, nrep=MAX_OBJ, rep_row=noo),
                opt.pack_seg(W1, t["w1"], K=ENC, chained=True),
                opt.pack_seg(W1, t["w1t"], K=HID, chained=True, transposed=True),
                opt.pack_seg(W2, t["w2"], K=HID, chained=True),
                opt.pack_seg(W2, t["w2t"], K=HID, chained=True, transposed=True)]
        if self.double:
            for k, p in (("b1", n.hidden_layer.bias), ("b2", n.hidden_layer_2.bias),
                         ("wout", n.output_layer.weight), ("bout", n.output_layer.bias)):
                segs.append(opt.pack_seg(p.reshape(-1), t[k], f32=True))
        self._segs[dst] = segs
        return segs

    def refresh(self, stream=None):
        """Re-pack every image set from the f32 parameters (eager: initial packs, loads, the DP path)."""
        src = self.src()
        for t in self.sets:
            _abi.check(self.L.asvrl_mlp_pack(C.byref(src), C.byref(t["w"]), _abi.stream_ptr(stream)),
                       "asvrl_mlp_pack", self.L)
            if self.double:
                n = self.net
                with torch.no_grad():
                    for k, p in (("b1", n.hidden_layer.bias), ("b2", n.hidden_layer_2.bias),
                                 ("wout", n.output_layer.weight), ("bout", n.output_layer.bias)):
                        t[k].copy_(p.reshape(-1))


def _rows(x):
    """(pointer base tensor, row stride in floats) of a row-major f32 view."""
    assert x.dtype == torch.float32 and x.stride(-1) == 1
    return x, x.stride(0)


def mlp_encode(pack, x, F, G=None, act=None, xb=None, stream=None):
    """F = observation_processor(x) [n][256]; G = action_encoder(act) [n][128]; xb = bf16 x[:, :32]."""
    x, ldx = _rows(x)
    io = _abi.AsvMlpIO()
    io.x, io.ldx, io.n = x.data_ptr(), ldx, x.shape[0]
    io.F, io.G, io.xb = _p(F), _p(G), _p(xb)
    if act is not None:
        io.act, io.lda = act.data_ptr(), act.stride(0)
    _abi.check(pack.L.asvrl_mlp_encode(C.byref(pack.w), C.byref(io), _abi.stream_ptr(stream)),
               "asvrl_mlp_encode", pack.L)


def actor_forward(pack, x, a_out, stream=None):
    """Actor.forward(x) -> a_out [n][2] f32 (no saved activations)."""
    x, ldx = _rows(x)
    io = _abi.AsvMlpIO()
    io.x, io.ldx, io.n = x.data_ptr(), ldx, x.shape[0]
    io.a_out, io.ld_aout = a_out.data_ptr(), a_out.stride(0)
    _abi.check(pack.L.asvrl_actor_forward(C.byref(pack.w), C.byref(io), MODE_FWD, _abi.stream_ptr(stream)),
               "asvrl_actor_forward", pack.L)


def actor_act(pack, x, actions64, step_dev, steps_per_count, total, fraction, initial, final, seed, stream=None):
    """Epsilon-greedy batched act (agent.py:207-225) into f64 actions [n][2]."""
    x, ldx = _rows(x)
    io = _abi.AsvMlpIO()
    io.x, io.ldx, io.n = x.data_ptr(), ldx, x.shape[0]
    io.a_out64 = actions64.data_ptr()
    io.step_dev = step_dev.data_ptr()
    io.eps_steps_per_count, io.eps_total, io.eps_fraction = float(steps_per_count), float(total), float(fraction)
    io.eps_initial, io.eps_final, io.seed = float(initial), float(final), int(seed) & 0xFFFFFFFFFFFFFFFF
    _abi.check(pack.L.asvrl_actor_forward(C.byref(pack.w), C.byref(io), MODE_ACT, _abi.stream_ptr(stream)),
               "asvrl_actor_forward(act)", pack.L)


class ActorBuffers:
    """Saved activations and backward outputs of one Actor training pass over B rows (operand dtype
    of the build, see MlpPack)."""

    def __init__(self, B, device, operands="bf16"):
        bf = dict(dtype=_abi.operand_dtype(operands), device=device)
        f = dict(dtype=torch.float32, device=device)
        self.B = B
        self.xb = torch.empty(B, OBSK, **bf)
        self.h0 = torch.empty(B, ENC, **bf)
        self.h1 = torch.empty(B, HID, **bf)
        self.h2 = torch.empty(B, HID, **bf)
        self.pre = torch.empty(B, 2, **f)
        self.a_out = torch.empty(B, 2, **f)
        self.dA = torch.empty(B, 2, **f)
        self.dout = torch.empty(B, 2, **f)
        self.dz2 = torch.empty(B, HID, **bf)
        self.dz1 = torch.empty(B, HID, **bf)
        self.dz0 = torch.empty(B, ENC, **bf)

    def io(self, x=None):
        io = _abi.AsvMlpIO()
        if x is not None:
            x, ldx = _rows(x)
            io.x, io.ldx = x.data_ptr(), ldx
        io.n = self.B
        io.xb, io.h0, io.h1, io.h2, io.pre = (self.xb.data_ptr(), self.h0.data_ptr(), self.h1.data_ptr(),
                                              self.h2.data_ptr(), self.pre.data_ptr())
        io.a_out, io.ld_aout = self.a_out.data_ptr(), 2
        io.dA, io.dout = self.dA.data_ptr(), self.dout.data_ptr()
        io.dz2, io.dz1, io.dz0 = self.dz2.data_ptr(), self.dz1.data_ptr(), self.dz0.data_ptr()
        return io


def actor_train_forward(pack, x, bufs, stream=None):
    io = bufs.io(x)
    _abi.check(pack.L.asvrl_actor_forward(C.byref(pack.w), C.byref(io), MODE_TRAIN, _abi.stream_ptr(stream)),
               "asvrl_actor_forward(train)", pack.L)
    return bufs.a_out


def actor_backward(pack, bufs, stream=None):
    """bufs.dA -> dout, dz2, dz1, dz0 (pre-activation gradients of every Actor layer)."""
    io = bufs.io()
    _abi.check(pack.L.asvrl_actor_backward(C.byref(pack.w), C.byref(io), _abi.stream_ptr(stream)),
               "asvrl_actor_backward", pack.L)


class ActorGrads:
    """Workspace of asvrl_actor_grads for one ActorBuffers (B rows): the split slabs, the arrival
    counters (zero, and left zero by every launch) and the squared-norm partials for asvrl_adam_step."""

    def __init__(self, B, device, operands="bf16"):
        self.L = _abi.lib(operands)
        self.work = torch.empty(int(self.L.asvrl_actor_grads_workspace(B)), dtype=torch.float32, device=device)
        # arrival counters: zero, and left zero by every launch
        self.counters = torch.zeros(int(self.L.asvrl_actor_grads_counters()), dtype=torch.int32, device=device)
        self.nparts = int(self.L.asvrl_actor_grads_norm_parts())
        self.norm_parts = torch.zeros(self.nparts, dtype=torch.float64, device=device)


def actor_grads(ws, bufs, actor, tile_loss=None, loss_out=None, step=None, norm=True, stream=None):
    """Every .grad of `actor` (hidden_layer, hidden_layer_2, output_layer, both observation encoders, whose
    four gradients must be contiguous: FusedAdam / FlatGrads) from bufs' backward outputs and saved
    activations, the loss sum(tile_loss) -> loss_out, the norm partials (ws.norm_parts, for
    FusedAdam.step_prenormed) and step += 1, in ONE launch (asvrl_actor_grads; agent.py:424-426)."""
    se, oe = actor.self_encoder[0], actor.object_encoder[0]
    gs = [se.weight.grad, se.bias.grad, oe.weight.grad, oe.bias.grad]
    if not all(gs[k].data_ptr() + 4 * gs[k].numel() == gs[k + 1].data_ptr() for k in range(3)):
        raise RuntimeError("actor_grads needs the encoder gradients contiguous (FusedAdam / FlatGrads)")
    io = _abi.AsvActorGradIO()
    io.xb, io.h0, io.h1, io.h2, io.dout = (bufs.xb.data_ptr(), bufs.h0.data_ptr(), bufs.h1.data_ptr(),
                                           bufs.h2.data_ptr(), bufs.dout.data_ptr())
    io.dz2, io.dz1, io.dz0 = bufs.dz2.data_ptr(), bufs.dz1.data_ptr(), bufs.dz0.data_ptr()
    io.B = bufs.B
    if tile_loss is not None and loss_out is not None:
        io.n_loss, io.tile_loss, io.loss_out = tile_loss.numel(), tile_loss.data_ptr(), loss_out.data_ptr()
    h1l, h2l, ol = actor.hidden_layer, actor.hidden_layer_2, actor.output_layer
    io.w1_grad, io.b1_grad = h1l.weight.grad.data_ptr(), h1l.bias.grad.data_ptr()
    io.w2_grad, io.b2_grad = h2l.weight.grad.data_ptr(), h2l.bias.grad.data_ptr()
    io.wo_grad, io.bo_grad = ol.weight.grad.data_ptr(), ol.bias.grad.data_ptr()
    io.enc_grad = gs[0].data_ptr()
    io.norm_parts = ws.norm_parts.data_ptr() if norm else None
    io.step = _p(step)
    io.work, io.work_floats, io.counters = ws.work.data_ptr(), ws.work.numel(), ws.counters.data_ptr()
    _abi.check(ws.L.asvrl_actor_grads(C.byref(io), _abi.stream_ptr(stream)), "asvrl_actor_grads", ws.L)


def encoder_fold(dw, db, net, accumulate=False, stream=None):
    """256 x 32 encoder-image gradient -> self_encoder / object_encoder .grad."""
    se, oe = net.self_encoder[0], net.object_encoder[0]
    _abi.check(_abi.lib().asvrl_encoder_fold(dw.data_ptr(), db.data_ptr(), se.weight.grad.data_ptr(),
                                             se.bias.grad.data_ptr(), oe.weight.grad.data_ptr(),
                                             oe.bias.grad.data_ptr(), int(accumulate), _abi.stream_ptr(stream)),
               "asvrl_encoder_fold")


def small_wgrad(dz, x, dw, db, work, accumulate=False, stream=None):
    """dw (M, K) <- dz^T x, db <- dz.sum(0) for f32 dz (R, M) and a small f32 x (R, K <= 4)."""
    R, M = dz.shape
    K = x.shape[1]
    _abi.check(_abi.lib().asvrl_small_wgrad(dz.data_ptr(), dz.stride(0), x.data_ptr(), x.stride(0), R, M, K,
                                            dw.data_ptr(), _p(db), int(accumulate), work.data_ptr(), work.numel(),
                                            _abi.stream_ptr(stream)), "asvrl_small_wgrad")
