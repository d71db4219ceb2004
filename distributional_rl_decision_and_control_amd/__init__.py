"""MI355X-native rfarl training hot path: vectorised ASV marine env + distributional
Bellman update on gfx950 kernels (libasvrl.so), behind rfarl's Python surfaces.

Import surfaces mirror the reference package (rfarl/rfarl/...):
  envs.marinenav.env.MarineNavEnv3, agent.Agent, policy.trainer.Trainer,
plus the batched fast path vec_env.VecMarineNavEnv / vec_trainer.VecTrainer.
"""
__version__ = "0.1.0"
