"""ctypes binding of libasvrl.so (include/asvrl.h).

The product path has exactly one compute backend: the gfx950 kernels in this library.
`lib()` raises if the library is missing or was built for another ABI; nothing falls back
to a CPU implementation.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ASVRL_LIB", os.path.join(HERE, "lib", "libasvrl.so"))  # override: A/B variants
# the same sources built with f32 learner operands (the parity build; asvrl_operand_bytes() == 4)
LIB_PATH_F32 = os.path.join(HERE, "lib", "libasvrl_f32.so")
OPERANDS = {"bf16": (LIB_PATH, 2), "f32": (LIB_PATH_F32, 4)}
ABI_VERSION = 26

SELF_DIM, OBJ_DIM, MAX_OBJ = 7, 5, 5
OBS_DIM = 40   # self 7 | objects 25 | mask 5 | pad 3
TR_DIM = 88    # obs 40 | next obs 40 | action 2 | reward | done | pad 4
PER_DIM = 48   # obs 40 | action | reward | nonterminal | timestep (i32) | pad 4

# robot state fields (enum AsvRobotField)
F_X, F_Y, F_THETA, F_VR0, F_VR1, F_VR2, F_V0, F_V1, F_V2, F_TL, F_TR, F_LP, F_RP, F_GX, F_GY, F_PHI, F_RET = range(17)
NUM_FIELDS = 17

FLAG_DEACTIVATED, FLAG_COLLISION, FLAG_REACH_GOAL, FLAG_COLREGS = 1, 2, 4, 8

INFO_NORMAL, INFO_TOO_LONG, INFO_COLLISION, INFO_REACH_GOAL, INFO_DEACT_COLLISION, INFO_DEACT_GOAL = range(6)
INFO_ABSENT = 255
INFO_STRINGS = {
    INFO_NORMAL: "normal",
    INFO_TOO_LONG: "too long episode",
    INFO_COLLISION: "collision",
    INFO_REACH_GOAL: "reach goal",
    INFO_DEACT_COLLISION: "deactivated after collision",
    INFO_DEACT_GOAL: "deactivated after reaching goal",
}

_HYDRO = ["xDotU", "yDotV", "yDotR", "nDotR", "nDotV", "xU", "xUU", "yV", "yVV", "yR", "yRV", "yVR", "yRR",
          "nR", "nRR", "nV", "nVV", "nRV", "nVR"]


class AsvParams(C.Structure):
    _fields_ = ([("dt", C.c_double), ("N", C.c_int32), ("episode_limit", C.c_int32),
                 ("length", C.c_double), ("width", C.c_double), ("r", C.c_double), ("goal_dis", C.c_double),
                 ("min_thrust", C.c_double), ("max_thrust", C.c_double), ("m", C.c_double), ("Izz", C.c_double)]
                + [(n, C.c_double) for n in _HYDRO]
                + [("P", C.c_double * 9), ("left_thrust_change", C.c_double * 5),
                   ("right_thrust_change", C.c_double * 5), ("range", C.c_double), ("angle", C.c_double),
                   ("pos_std", C.c_double), ("vel_std", C.c_double), ("r_kappa", C.c_double),
                   ("r_mean_ratio", C.c_double), ("max_obj_num", C.c_int32), ("_pad0", C.c_int32),
                   ("timestep_penalty", C.c_double), ("COLREGs_penalty", C.c_double),
                   ("collision_penalty", C.c_double), ("goal_reward", C.c_double), ("core_r", C.c_double)])


class AsvEnvState(C.Structure):
    _fields_ = [("n_envs", C.c_int32), ("max_robots", C.c_int32), ("max_obs", C.c_int32), ("max_cores", C.c_int32),
                ("rs", C.c_void_p), ("rflags", C.c_void_p), ("n_robots", C.c_void_p), ("n_obs", C.c_void_p),
                ("n_cores", C.c_void_p), ("ep_ts", C.c_void_p), ("obstacles", C.c_void_p), ("cores", C.c_void_p),
                ("robot_params", C.c_void_p)]


class AsvStepCtl(C.Structure):
    _fields_ = [("is_continuous", C.c_int32), ("do_dynamics", C.c_int32), ("trainer_deactivate", C.c_int32),
                ("noise_mode", C.c_int32), ("seed", C.c_uint64), ("counter", C.c_uint64),
                ("counter_dev", C.c_void_p), ("gamma", C.c_double), ("env_mask", C.c_void_p)]


class AsvStepOut(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("obs64", C.c_void_p), ("obj_cnt", C.c_void_p), ("reward", C.c_void_p),
                ("done", C.c_void_p), ("info", C.c_void_p), ("env_done", C.c_void_p), ("stats", C.c_void_p)]


class AsvResetCfg(C.Structure):
    _fields_ = [("num_robots", C.c_int32), ("num_obs", C.c_int32), ("num_cores", C.c_int32), ("_pad0", C.c_int32),
                ("min_start_goal_dis", C.c_double), ("width", C.c_double), ("height", C.c_double),
                ("clear_r", C.c_double), ("obs_r_lo", C.c_double), ("obs_r_hi", C.c_double), ("v_lo", C.c_double),
                ("v_hi", C.c_double), ("v_rel_max", C.c_double), ("p_rel", C.c_double)]


class AsvEnvLaunch(C.Structure):
    _fields_ = [("layout", C.c_int32), ("block", C.c_int32), ("envs_per_block", C.c_int32), ("max_groups", C.c_int32)]


ENV_LAYOUT_AUTO, ENV_LAYOUT_PAIRS, ENV_LAYOUT_SWEEP = 0, 1, 2


class AsvCriticWeights(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("wc_frag", "w1_frag", "w2_frag", "w2t_frag", "w1t_frag", "bc", "b1", "b2",
                                          "wo", "bo", "self_w", "self_b", "obj_w", "obj_b", "ae_w", "ae_b")]


class AsvCriticActs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("cos", "h0", "dzc", "h1g", "dz1", "h2", "dz2", "dq", "wout_part")]


class AsvCriticParts(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("cos_emb", "hidden", "hidden2", "out", "enc", "aenc")]


# (name, restype, argtypes) of every exported entry point, mirroring include/asvrl.h
_VP, _I32, _I64, _U64, _F, _D = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_double
class AsvCriticIO(C.Structure):
    _fields_ = [("F", _VP), ("G", _VP), ("obs", _VP), ("ld_obs", _I64), ("act", _VP), ("ld_act", _I64), ("xb", _VP),
                ("taus", _VP), ("B", _I32), ("N", _I32), ("Np", _I32), ("kappa", C.c_float),
                ("q_targets", _VP), ("q_next", _VP), ("rewards", _VP), ("dones", _VP), ("ld_rd", _I64),
                ("gamma", C.c_float), ("dq", C.c_float), ("q", _VP), ("row_loss", _VP), ("dF", _VP), ("dG", _VP),
                ("dzF", _VP), ("dzG", _VP), ("w_ae", _VP), ("dA", _VP), ("tile_loss", _VP),
                ("loss_scale", C.c_float)]


IQN_MAX_ACTIONS = 32


class AsvIqnHead(C.Structure):
    _fields_ = [("wo_frag", _VP), ("wo", _VP), ("bo", _VP), ("n_actions", _I32)]


class AsvIqnIO(C.Structure):
    _fields_ = [("F", _VP), ("obs", _VP), ("ld_obs", _I64), ("xb", _VP), ("taus", _VP), ("B", _I32), ("N", _I32),
                ("Np", _I32), ("kappa", C.c_float), ("q_next", _VP), ("actions", _VP), ("rewards", _VP),
                ("dones", _VP), ("ld_rd", _I64),
                ("gamma", C.c_float), ("q", _VP), ("row_loss", _VP), ("dzF", _VP), ("dz_out", _VP),
                ("tile_loss", _VP), ("loss_scale", C.c_float), ("act_out", _VP), ("ld_act", _I64),
                ("step_dev", _VP), ("eps_steps_per_count", _D), ("eps_total", _D), ("eps_fraction", _D),
                ("eps_initial", _D), ("eps_final", _D), ("seed", _U64)]


MAX_SUM_SEGS = 24


SUM_PLAIN, SUM_FOLD_ENCODERS = 0, 1


MAX_WGRAD_SEGS = 24
MAX_PACK_SEGS = 16


class AsvPackSeg(C.Structure):
    _fields_ = [("flat_off", _I64), ("image", _VP), ("rows", _I32), ("cols", _I32), ("K", _I32), ("chained", _I32),
                ("transposed", _I32), ("f32", _I32), ("row0", _I32), ("col0", _I32), ("nrep", _I32),
                ("rep_row", _I32), ("rep_col", _I32), ("reserved", _I32)]
WGRAD_MFMA, WGRAD_VEC, WGRAD_SMALL = 0, 1, 2


class AsvWgradSeg(C.Structure):
    _fields_ = [("dz", _VP), ("ldz", _I64), ("x", _VP), ("ldx", _I64), ("R", _I32), ("M", _I32), ("K", _I32),
                ("kind", _I32), ("partial", _VP), ("partial_floats", _I64)]


class AsvActorGradIO(C.Structure):
    _fields_ = [(n, _VP) for n in ("xb", "h0", "h1", "h2", "dout", "dz2", "dz1", "dz0")] + \
               [("B", _I32), ("n_loss", _I32)] + \
               [(n, _VP) for n in ("tile_loss", "loss_out", "w1_grad", "b1_grad", "w2_grad", "b2_grad", "wo_grad",
                                   "bo_grad", "enc_grad", "norm_parts", "step", "work")] + \
               [("work_floats", _I64), ("counters", _VP)]


class AsvPartialSum(C.Structure):
    _fields_ = [("partial", _VP), ("dw", _VP), ("db", _VP), ("groups", _I32), ("nw", _I32), ("nb", _I32),
                ("accumulate", _I32), ("stride", _I32), ("boff", _I32), ("mode", _I32), ("norm", _I32)]


class AsvMlpSrc(C.Structure):
    _fields_ = [(n, _VP) for n in ("self_w", "self_b", "obj_w", "obj_b", "w1", "w2", "ae_w")]


class AsvMlpWeights(C.Structure):
    _fields_ = [(n, _VP) for n in ("enc_frag", "b_enc", "w1_frag", "w2_frag", "w2t_frag", "w1t_frag", "b1", "b2",
                                   "wout", "bout", "ae_frag", "b_ae")] + [("out_scale", C.c_float)]


class AsvMlpIO(C.Structure):
    _fields_ = [("x", _VP), ("ldx", _I64), ("act", _VP), ("lda", _I64), ("n", _I32), ("F", _VP), ("G", _VP),
                ("xb", _VP), ("a_out", _VP), ("ld_aout", _I64), ("a_out64", _VP), ("pre", _VP), ("h0", _VP),
                ("h1", _VP), ("h2", _VP), ("dA", _VP), ("dout", _VP), ("dz2", _VP), ("dz1", _VP), ("dz0", _VP),
                ("step_dev", _VP), ("eps_steps_per_count", _D), ("eps_total", _D), ("eps_fraction", _D),
                ("eps_initial", _D), ("eps_final", _D), ("seed", _U64)]


class AsvSampleArgs(C.Structure):
    _fields_ = [("ring", _VP), ("capacity", _I64), ("ring_state", _VP), ("seed", _U64), ("counter", _U64),
                ("counter_dev", _VP), ("guard", _I64), ("B", _I32), ("tau_sets", _I32), ("tau_n", _I32),
                ("_pad0", _I32), ("out", _VP), ("taus", _VP)]


class AsvPer(C.Structure):
    _fields_ = [("rows", _VP), ("tree", _VP), ("state", _VP), ("t", _VP), ("maxp", _VP), ("dirty", _VP),
                ("capacity", _I64), ("tree_leaves", _I64), ("stride", _I32), ("n_step", _I32), ("discount", _D),
                ("priority_weight", C.c_float), ("priority_exponent", C.c_float), ("deferred", _I32),
                ("_pad0", _I32)]


MAX_NOISY_SEGS = 16


class AsvNoisySeg(C.Structure):
    _fields_ = [(n, _VP) for n in ("mu", "sigma", "eps", "out", "dout", "dmu", "dsigma")]


class AsvNoisySegs(C.Structure):
    _fields_ = [("n", _I32), ("_pad0", _I32), ("off", _I64 * (MAX_NOISY_SEGS + 1)),
                ("seg", AsvNoisySeg * MAX_NOISY_SEGS)]


class AsvRainbowHeadIO(C.Structure):
    _fields_ = [("v", _VP), ("ldv", _I64), ("a", _VP), ("lda", _I64), ("N", _I32), ("atoms", _I32),
                ("actions_n", _I32), ("_pad0", _I32), ("support", _VP), ("act_out", _VP), ("ld_act", _I64),
                ("act_idx", _VP), ("step_dev", _VP), ("eps_steps_per_count", _D), ("eps_total", _D),
                ("eps_fraction", _D), ("eps_initial", _D), ("eps_final", _D), ("seed", _U64), ("p_out", _VP),
                ("actions", _VP), ("weights", _VP), ("ld_rd", _I64), ("m", _VP), ("loss", _VP), ("dv", _VP),
                ("da", _VP), ("grad_scale", C.c_float), ("_pad1", _I32)]



class AsvRainbowSrc(C.Structure):
    _fields_ = [(n, _VP) for n in ("self_w", "self_b", "obj_w", "obj_b", "w_v1", "b_v1", "w_a1", "b_a1", "w_v2", "b_v2",
                                   "w_a2", "b_a2", "w_vo", "b_vo", "w_ao", "b_ao")]


RAINBOW_IMG_FIELDS = ("enc", "v1", "a1", "v2", "a2", "vo", "mo", "ao")
RAINBOW_BIAS_FIELDS = ("b_enc", "b_v1p", "b_a1p", "b_v2p", "b_a2p", "b_vop", "b_mop", "b_aop")
RAINBOW_IMGT_FIELDS = ("vot", "mot", "aot", "v2t", "a2t", "v1t", "a1t")


class AsvRainbowImg(C.Structure):   # also AsvRainbowImgOut (same layout)
    _fields_ = [(n, _VP) for n in RAINBOW_IMG_FIELDS + RAINBOW_BIAS_FIELDS + RAINBOW_IMGT_FIELDS]


class AsvRainbowNetIO(C.Structure):
    _fields_ = [("x", _VP), ("ldx", _I64), ("N", _I32), ("_pad0", _I32), ("support", _VP), ("act_out", _VP),
                ("ld_act", _I64), ("act_idx", _VP), ("step_dev", _VP), ("eps_steps_per_count", _D), ("eps_total", _D),
                ("eps_fraction", _D), ("eps_initial", _D), ("eps_final", _D), ("seed", _U64), ("p_out", _VP),
                ("actions", _VP), ("weights", _VP), ("ld_rd", _I64), ("m", _VP), ("grad_scale", _F), ("_pad1", _I32),
                ("loss", _VP)] + [(n, _VP) for n in ("xb", "f", "hv1", "ha1", "hv2", "ha2", "dzv", "dza", "dz2v",
                                                     "dz2a", "dz1v", "dz1a", "dzf")]


EXPORTS = [
    ("asvrl_env_step", C.c_int, [C.POINTER(AsvParams), C.POINTER(AsvEnvState), _VP, _VP, C.POINTER(AsvStepCtl),
                                 C.POINTER(AsvStepOut), _VP]),
    ("asvrl_env_step_ex", C.c_int, [C.POINTER(AsvParams), C.POINTER(AsvEnvState), _VP, _VP, C.POINTER(AsvStepCtl),
                                    C.POINTER(AsvStepOut), C.POINTER(AsvEnvLaunch), _VP]),
    ("asvrl_env_reset", C.c_int, [C.POINTER(AsvParams), C.POINTER(AsvEnvState), C.POINTER(AsvResetCfg), _VP, _U64,
                                  _U64, _VP, _VP]),
    ("asvrl_env_reset_observe", C.c_int, [C.POINTER(AsvParams), C.POINTER(AsvEnvState), C.POINTER(AsvResetCfg), _VP,
                                          _U64, _U64, _VP, C.POINTER(AsvStepCtl), C.POINTER(AsvStepOut), _VP]),
    ("asvrl_current_field", C.c_int, [_VP, _I32, _D, _VP, _I32, _VP, _VP]),
    ("asvrl_quantile_huber", C.c_int, [_VP, _VP, _VP, _I32, _I32, _I32, _F, _F, _VP, _VP, _VP, _VP]),
    ("asvrl_c51_project", C.c_int, [_VP, _VP, _VP, _VP, _I32, _I32, _F, _F, _F, _F, _VP, _VP]),
    ("asvrl_c51_project_ex", C.c_int, [_VP, _VP, C.c_int64, _VP, C.c_int64, _VP, _I32, _I32, _F, _F, _F, _F, _VP,
                                       _VP]),
    ("asvrl_critic_pack", C.c_int, [_VP, _VP, _VP, C.POINTER(AsvCriticWeights), _VP]),
    ("asvrl_critic_forward", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvCriticIO), _VP]),
    ("asvrl_critic_train", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvCriticIO), C.POINTER(AsvCriticActs),
                                     _VP]),
    ("asvrl_critic_actor_grad", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvCriticIO), _VP]),
    ("asvrl_iqn_pack", C.c_int, [_VP, _VP, _VP, _VP, C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), _VP]),
    ("asvrl_iqn_forward_max", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO), _VP]),
    ("asvrl_iqn_train", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO),
                                  C.POINTER(AsvCriticActs), _VP]),
    ("asvrl_iqn_act", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO), _VP]),
    ("asvrl_replay_push", C.c_int, [_VP, _VP, _VP, _VP, _I32, _VP, _VP, _I32, _VP, _I64, _VP, _VP, _VP]),
    ("asvrl_replay_push_ex", C.c_int, [_VP, _VP, _VP, _VP, _I32, _I64, _VP, _VP, _I32, _VP, _I64, _VP, _VP, _VP,
                                       _VP, _VP]),
    ("asvrl_replay_sample", C.c_int, [_VP, _I64, _VP, _VP, _I32, _U64, _U64, _VP, _I64, _VP, _VP, _VP, _I32, _I32,
                                      _VP]),
    ("asvrl_replay_write_rows", C.c_int, [_VP, _VP, _I32, _VP, _VP]),
    ("asvrl_per_push", C.c_int, [C.POINTER(AsvPer), _VP, _VP, _VP, _I32, _VP, _VP, _I32, _VP]),
    ("asvrl_per_sample", C.c_int, [C.POINTER(AsvPer), _I32, _VP, _U64, _U64, _VP, _VP, _VP, _VP]),
    ("asvrl_per_update", C.c_int, [C.POINTER(AsvPer), _VP, _VP, _I32, _I32, _VP]),
    ("asvrl_per_push_ex", C.c_int, [C.POINTER(AsvPer), _VP, _VP, _VP, _I32, _VP, _VP, _I32, _VP, _VP]),
    ("asvrl_per_update_ex", C.c_int, [C.POINTER(AsvPer), _VP, _VP, _I32, _I32, _VP, _VP, _VP]),
    ("asvrl_per_sample_ex", C.c_int, [C.POINTER(AsvPer), _I32, _VP, _U64, _U64, _VP, _VP, _VP, _VP, _VP]),
    ("asvrl_per_normalise", C.c_int, [_VP, _VP, _I32, _VP]),
    ("asvrl_noisy_compose", C.c_int, [C.POINTER(AsvNoisySegs), _I32, _VP]),
    ("asvrl_noisy_backward_norm_parts", _I32, [C.POINTER(AsvNoisySegs)]),
    ("asvrl_noisy_backward_norm", C.c_int, [C.POINTER(AsvNoisySegs), _VP, _VP]),
    ("asvrl_noisy_reset", C.c_int, [C.POINTER(AsvNoisySegs), _VP, _VP, _U64, _VP, _VP]),
    ("asvrl_rainbow_act", C.c_int, [C.POINTER(AsvRainbowHeadIO), _VP]),
    ("asvrl_rainbow_pick", C.c_int, [C.POINTER(AsvRainbowHeadIO), _VP]),
    ("asvrl_rainbow_loss", C.c_int, [C.POINTER(AsvRainbowHeadIO), _VP]),
    ("asvrl_rainbow_pack", C.c_int, [C.POINTER(AsvRainbowSrc), C.POINTER(AsvRainbowImg), _VP]),
    ("asvrl_rainbow_net_act", C.c_int, [C.POINTER(AsvRainbowImg), C.POINTER(AsvRainbowNetIO), _VP]),
    ("asvrl_rainbow_net_argmax", C.c_int, [C.POINTER(AsvRainbowImg), C.POINTER(AsvRainbowNetIO), _VP]),
    ("asvrl_rainbow_net_pick", C.c_int, [C.POINTER(AsvRainbowImg), C.POINTER(AsvRainbowNetIO), _VP]),
    ("asvrl_rainbow_net_train", C.c_int, [C.POINTER(AsvRainbowImg), C.POINTER(AsvRainbowNetIO), _VP]),
    ("asvrl_adam_clip", C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP, _F, _F, _F, _F, _F, _VP, _VP, _VP]),
    ("asvrl_linear_wgrad_workspace", _I64, [_I32, _I32]),
    ("asvrl_critic_wout_groups", _I32, [_I32, _I32]),
    ("asvrl_critic_fused_groups", _I32, [_I32, _I32]),
    ("asvrl_critic_fused_variant", _I32, [_I32]),
    ("asvrl_critic_train_fused", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvCriticIO),
                                           C.POINTER(AsvCriticParts), _VP]),
    ("asvrl_critic_train_fused_tq", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvCriticIO),
                                              C.POINTER(AsvCriticParts), C.POINTER(AsvCriticWeights),
                                              C.POINTER(AsvCriticIO), _VP]),
    ("asvrl_iqn_train_fused", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO),
                                        C.POINTER(AsvCriticParts), _VP]),
    ("asvrl_iqn_train_fused_tq", C.c_int, [C.POINTER(AsvCriticWeights), C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO),
                                           C.POINTER(AsvCriticParts), C.POINTER(AsvCriticWeights),
                                           C.POINTER(AsvIqnHead), C.POINTER(AsvIqnIO), _VP]),
    ("asvrl_linear_wgrad_groups", _I32, [_I32, _I32, _I32]),
    ("asvrl_linear_wgrad_vec_groups", _I32, [_I32]),
    ("asvrl_linear_wgrad_partial", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _I32, _VP, _I64, _VP, _VP]),
    ("asvrl_linear_wgrad_multi", C.c_int, [_VP, _I32, _VP, _VP]),
    ("asvrl_linear_wgrad_vec_partial", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _VP, _I64, _VP, _VP]),
    ("asvrl_small_wgrad_partial", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _I32, _VP, _I64, _VP, _VP]),
    ("asvrl_partial_sums", C.c_int, [_VP, _I32, _VP]),
    ("asvrl_partial_sums_norm", C.c_int, [_VP, _I32, _VP, _VP, _VP]),
    ("asvrl_partial_sums_norm_parts", _I32, [_VP, _I32]),
    ("asvrl_actor_grads_workspace", _I64, [_I32]),
    ("asvrl_actor_grads_counters", _I32, []),
    ("asvrl_actor_grads_norm_parts", _I32, []),
    ("asvrl_actor_grads", C.c_int, [C.POINTER(AsvActorGradIO), _VP]),
    ("asvrl_adam_step", C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP, _F, _F, _F, _F, _F, _VP, _VP, _I32, _VP]),
    ("asvrl_adam_step_pack", C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP, _F, _F, _F, _F, _F, _VP, _VP, _I32, _VP, _I32,
                                       _VP, _VP]),
    ("asvrl_linear_wgrad", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _I32, _VP, _VP, _I32, _VP, _I64, _VP]),
    ("asvrl_linear_wgrad_vec", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _VP, _VP, _I32, _VP, _I64, _VP]),
    ("asvrl_mlp_pack", C.c_int, [C.POINTER(AsvMlpSrc), C.POINTER(AsvMlpWeights), _VP]),
    ("asvrl_mlp_encode", C.c_int, [C.POINTER(AsvMlpWeights), C.POINTER(AsvMlpIO), _VP]),
    ("asvrl_actor_forward", C.c_int, [C.POINTER(AsvMlpWeights), C.POINTER(AsvMlpIO), _I32, _VP]),
    ("asvrl_actor_backward", C.c_int, [C.POINTER(AsvMlpWeights), C.POINTER(AsvMlpIO), _VP]),
    ("asvrl_learn_prologue", C.c_int, [C.POINTER(AsvSampleArgs), C.POINTER(AsvMlpWeights), C.POINTER(AsvMlpIO),
                                       C.POINTER(AsvMlpWeights), _VP, _VP]),
    ("asvrl_encoder_fold", C.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _I32, _VP]),
    ("asvrl_small_wgrad", C.c_int, [_VP, _I64, _VP, _I64, _I32, _I32, _I32, _VP, _VP, _I32, _VP, _I64, _VP]),
    ("asvrl_last_error", C.c_char_p, []),
    ("asvrl_abi_version", C.c_int, []),
    ("asvrl_operand_bytes", C.c_int32, []),
    ("asvrl_struct_sizes", None, [C.c_void_p]),
]

_libs = {}


class AsvrlError(RuntimeError):
    pass


def lib(operands="bf16"):
    """Load libasvrl.so (operands="bf16", the product) or libasvrl_f32.so (operands="f32", the
    f32-operand parity build of the same sources), built by __graft_entry__.build /
    `python -m ...build`. Raises if absent: there is no CPU fallback."""
    L = _libs.get(operands)
    if L is not None:
        return L
    if operands not in OPERANDS:
        raise ValueError(f"operands must be one of {sorted(OPERANDS)}")
    path, nbytes = OPERANDS[operands]
    if not os.path.exists(path):
        raise AsvrlError(f"{os.path.basename(path)} not found at {path}: build it with "
                         "`python -m distributional_rl_decision_and_control_amd.build` (hipcc, gfx950). "
                         "There is no CPU fallback.")
    L = C.CDLL(path)
    for name, res, args in EXPORTS:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    v = L.asvrl_abi_version()
    if v != ABI_VERSION:
        raise AsvrlError(f"{os.path.basename(path)} ABI {v} != expected {ABI_VERSION}; rebuild")
    if L.asvrl_operand_bytes() != nbytes:
        raise AsvrlError(f"{path}: operand element of {L.asvrl_operand_bytes()} bytes, expected {nbytes}")
    _libs[operands] = L
    return L


def operand_dtype(operands="bf16"):
    """torch dtype of the weight images / saved activations of a learner-kernel build."""
    import torch
    return {"bf16": torch.bfloat16, "f32": torch.float32}[operands]


def check(rc, what="", L=None):
    if rc != 0:
        msg = (L if L is not None else lib()).asvrl_last_error().decode(errors="replace")
        raise AsvrlError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Raw device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def params_from(robot=None, env=None, max_obj_num=5, episode_limit=1000):
    """AsvParams from a Robot-like object (wamv.py:45-125 attribute names) and env rewards.

    P = inv(A^T A) A^T is evaluated with the reference's own numpy matrix expression
    (wamv.py:267-271) so the kernel multiplies by the exact same f64 constants."""
    p = AsvParams()
    src = robot if robot is not None else _DefaultRobot()
    p.dt = float(src.dt)
    p.N = int(src.N)
    p.episode_limit = int(episode_limit)
    p.length, p.width = float(src.length), float(src.width)
    p.r = float(src.r)
    p.goal_dis = float(src.goal_dis)
    p.min_thrust, p.max_thrust = float(src.min_thrust), float(src.max_thrust)
    p.m, p.Izz = float(src.m), float(src.Izz)
    for n in _HYDRO:
        setattr(p, n, float(getattr(src, n)))
    import warnings
    warnings.filterwarnings("ignore", category=PendingDeprecationWarning, message=".*matrix subclass.*")
    M_RB = np.matrix([[src.m, 0.0, 0.0], [0.0, src.m, 0.0], [0.0, 0.0, src.Izz]])
    M_A = -1.0 * np.matrix([[src.xDotU, 0.0, 0.0], [0.0, src.yDotV, src.yDotR], [0.0, src.nDotV, src.nDotR]])
    A = M_RB + M_A
    P = np.asarray(np.linalg.inv(A.transpose() * A) * A.transpose(), dtype=np.float64).reshape(-1)
    for k in range(9):
        p.P[k] = float(P[k])
    for k in range(5):
        p.left_thrust_change[k] = float(src.left_thrust_change[k])
        p.right_thrust_change[k] = float(src.right_thrust_change[k])
    per = src.perception if hasattr(src, "perception") else src
    p.range, p.angle = float(per.range), float(per.angle)
    p.pos_std, p.vel_std = float(per.pos_std), float(per.vel_std)
    p.r_kappa, p.r_mean_ratio = float(per.r_kappa), float(per.r_mean_ratio)
    p.max_obj_num = int(getattr(per, "max_obj_num", max_obj_num))
    e = env if env is not None else _DefaultEnv()
    p.timestep_penalty = float(e.timestep_penalty)
    p.COLREGs_penalty = float(e.COLREGs_penalty)
    p.collision_penalty = float(e.collision_penalty)
    p.goal_reward = float(e.goal_reward)
    p.core_r = float(e.r)
    return p


class _DefaultRobot:
    """Reference defaults (wamv.py:22-25,45-125)."""
    dt, N, length, width = 0.05, 10, 5.0, 2.5
    r = 0.5 * np.sqrt(5.0 ** 2 + 2.5 ** 2)
    goal_dis, min_thrust, max_thrust = 2.0, -500.0, 1000.0
    m, Izz = 400, 450
    xDotU, yDotV, yDotR, nDotR, nDotV = 20, 0, 0, -980, 0
    xU, xUU, yV, yVV, yR, yRV, yVR, yRR = -100, -150, -100, -150, 0, 0, 0, 0
    nR, nRR, nV, nVV, nRV, nVR = -980, -950, 0, 0, 0, 0
    left_thrust_change = right_thrust_change = [0.0, -500.0, -1000.0, 500.0, 1000.0]
    range, angle, max_obj_num = 20.0, 2 * np.pi, 5
    pos_std, vel_std, r_kappa, r_mean_ratio = 0.05, 0.05, 1.0, 0.8


class _DefaultEnv:
    """Reference defaults (env.py:35,47-50)."""
    r = 0.5
    timestep_penalty, COLREGs_penalty, collision_penalty, goal_reward = -0.1, -0.1, -5.0, 10.0
