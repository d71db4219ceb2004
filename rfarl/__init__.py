"""`rfarl` import alias for the MI355X framework.

With this repository on PYTHONPATH, the reference's import paths --
rfarl.envs.marinenav.env.MarineNavEnv3, rfarl.agent.Agent, rfarl.policy.trainer.Trainer,
rfarl.utils.replay_buffer.ReplayBuffer, rfarl.policy.*_model, rfarl.scripts.train_RL_agents
-- resolve to distributional_rl_decision_and_control_amd, so the reference's training script
and config files drive the GPU path unchanged.
"""
import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = "distributional_rl_decision_and_control_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):
        return None


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith("rfarl."):
            return None
        tgt = _TARGET + fullname[len("rfarl"):]
        if importlib.util.find_spec(tgt) is None:
            return None
        spec = importlib.util.spec_from_loader(fullname, _AliasLoader(tgt),
                                               is_package=importlib.util.find_spec(tgt).submodule_search_locations is not None)
        return spec


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
