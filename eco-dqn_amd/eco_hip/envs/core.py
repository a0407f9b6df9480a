"""src/envs/core.py:3-10: make("SpinSystem", graph_generator, max_steps, **env_args)."""
from .spinsystem import SpinSystemFactory


def make(id, *args, **kwargs):
    if id == "SpinSystem":
        return SpinSystemFactory.get(*args, **kwargs)
    raise NotImplementedError()
