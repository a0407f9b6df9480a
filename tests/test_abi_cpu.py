"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every
entry point include/eco_hip.h declares (no compute calls without a GPU)."""
import os
import re
import ctypes

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "eco_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(eco_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from eco_hip import _lib
    declared = _declared()
    assert len(declared) >= 10
    missing = [s for s in declared if not hasattr(_lib.lib, s)]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared surface
    assert sorted(_lib.EXPORTS) == declared


def test_pure_queries_without_gpu():
    from eco_hip import _lib
    assert _lib.lib.eco_mpnn_param_count(7) == 58425
    assert _lib.lib.eco_mpnn_param_count(1) == 58425 - 6 * 64 - 6 * 63
    assert _lib.lib.eco_mpnn_packed_count() >= 58425
    from eco_hip.envs.batched import make_config
    from eco_hip.envs.utils import (DEFAULT_OBSERVABLES, RewardSignal, ExtraAction, OptimisationTarget,
                                    SpinBasis)
    cfg = make_config(200, 400, observables=DEFAULT_OBSERVABLES, reward_signal=RewardSignal.BLS,
                      extra_action=ExtraAction.NONE, optimisation_target=OptimisationTarget.CUT,
                      spin_basis=SpinBasis.SIGNED, norm_rewards=True, basin_reward=1 / 200)
    assert _lib.lib.eco_env_state_bytes(ctypes.byref(cfg), 8192) > 8192 * 200 * 8


def test_boundary_errors_map_to_reference_exceptions():
    import pytest
    from eco_hip.envs.batched import make_config
    from eco_hip.envs.utils import Observable, ExtraAction, OptimisationTarget
    with pytest.raises(NotImplementedError):   # factory has no ENERGY branch (score_solver.py:885)
        make_config(20, 40, extra_action=ExtraAction.NONE)
    with pytest.raises(AssertionError):        # spinsystem.py:116
        make_config(20, 40, observables=[Observable.TIME_SINCE_FLIP], extra_action=ExtraAction.NONE,
                    optimisation_target=OptimisationTarget.CUT)


def test_header_enums_match_reference_values():
    from eco_hip.envs import utils as u
    src = open(os.path.join(REPO, "include", "eco_hip.h")).read()
    for o in u.Observable:
        assert re.search(rf"ECO_OBS_{o.name}\s*=\s*{o.value}\b", src), o
    for r in u.RewardSignal:
        assert re.search(rf"ECO_REWARD_{r.name}\s*=\s*{r.value}\b", src), r
