"""Execute the reference's own `src/custom_env.py` and `src/environment.py`
(UNCHANGED, read as text from /root/reference) on top of the clean-room
minigrid / gymnasium restatement in this directory.

TEST INFRASTRUCTURE ONLY -- used by `tests/golden/make_golden.py` in the build
container to generate golden fixtures.  /root/reference does not exist on the
GPU box and nothing on the product path imports this module.

The source files are compiled from their .py text (never from the reference's
checked-in __pycache__), so exactly the published code runs.
"""
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = os.environ.get("MGX_REFERENCE_SRC", "/root/reference/src")


def _exec_module(name, path):
    with open(path, "r") as f:
        src = f.read()
    mod = types.ModuleType(name)
    mod.__file__ = path
    sys.modules[name] = mod
    exec(compile(src, path, "exec"), mod.__dict__)
    return mod


def load_reference():
    """Return (custom_env_module, environment_module)."""
    if HERE not in sys.path:
        sys.path.insert(0, HERE)
    sys.dont_write_bytecode = True
    if "custom_env" in sys.modules and "environment" in sys.modules:
        return sys.modules["custom_env"], sys.modules["environment"]
    ce = _exec_module("custom_env", os.path.join(REF_SRC, "custom_env.py"))
    env = _exec_module("environment", os.path.join(REF_SRC, "environment.py"))
    return ce, env


class Cfg(dict):
    """Attribute-and-item access config, standing in for the OmegaConf
    DictConfig the reference receives from Hydra (`single.yaml:20-28`)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v


def make_cfg(problem="multi", mission=5, size=8, num_objects=4, seed=42,
             see_through_walls=True, all_doors_open=False, obstacles=False,
             percent_obstacles=0.05, n_frames_stack=4):
    env = Cfg(problem=problem, mission=mission, all_doors_open=all_doors_open,
              size=size, num_objects=num_objects,
              see_through_walls=see_through_walls, obstacles=obstacles,
              percent_obstacles=percent_obstacles)
    alg = Cfg(n_frames_stack=n_frames_stack, recurrent=False)
    return Cfg(env=env, algorithm=alg, seed=seed, env_name="custom")
