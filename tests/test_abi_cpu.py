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


def test_set_kernel_paths_returns_previous_and_masks_unknown_bits():
    """eco_set_kernel_paths is host-only: the policy word the MPNN dispatcher reads (no GPU needed)."""
    from eco_hip import _lib
    prev = _lib.lib.eco_set_kernel_paths(0x7FFFFFFF)
    # the documented bits (NO_DENSE .. DENSE2_FWD); nothing else survives
    assert _lib.lib.eco_set_kernel_paths(prev) == 0x1F
    with _lib.kernel_paths(_lib.ECO_PATH_NO_PAIR):
        assert _lib.lib.eco_set_kernel_paths(_lib.ECO_PATH_NO_PAIR) == _lib.ECO_PATH_NO_PAIR
    assert _lib.lib.eco_set_kernel_paths(prev) == prev


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


def test_target_enums_and_config_validation():
    """OptimisationTarget values, and the C-side config check (eco_env_state_bytes returns 0 for a config
    eco_env_reset would reject): every set problem takes all 13 MAIN_OBSERVABLES; the cut scorers reject
    the validity-mask observables (a TypeError in the reference); ENERGY has no scorer."""
    import pytest
    from eco_hip import _lib
    from eco_hip.envs import utils as u
    from eco_hip.envs.batched import make_config
    src = open(os.path.join(REPO, "include", "eco_hip.h")).read()
    for t in u.OptimisationTarget:
        assert re.search(rf"ECO_TARGET_{t.name}\s*=\s*{t.value}\b", src), t
    kw = dict(reward_signal=u.RewardSignal.BLS, extra_action=u.ExtraAction.NONE, norm_rewards=True,
              basin_reward=1 / 20)
    for t in (u.OptimisationTarget.MIN_COVER, u.OptimisationTarget.MAX_IND_SET, u.OptimisationTarget.MAX_CLIQUE,
              u.OptimisationTarget.MIN_DOM_SET):
        cfg = make_config(20, 40, observables=u.MAIN_OBSERVABLES, optimisation_target=t, **kw)
        assert cfg.n_obs == 13 and _lib.obs_x_stride(cfg.n_obs) == 16
        assert _lib.lib.eco_env_state_bytes(ctypes.byref(cfg), 4) > 0, t
    for t in (u.OptimisationTarget.CUT, u.OptimisationTarget.MIN_CUT):
        with pytest.raises(TypeError):
            make_config(20, 40, observables=u.MAIN_OBSERVABLES, optimisation_target=t, **kw)
        cfg = make_config(20, 40, observables=u.DEFAULT_OBSERVABLES, optimisation_target=t, **kw)
        assert _lib.lib.eco_env_state_bytes(ctypes.byref(cfg), 4) > 0
        cfg.n_obs = 13                                   # bypass the Python check: the library rejects it too
        for i, o in enumerate(u.MAIN_OBSERVABLES):
            cfg.obs_ids[i] = o.value
        assert _lib.lib.eco_env_state_bytes(ctypes.byref(cfg), 4) == 0
    cfg = make_config(20, 40, optimisation_target=u.OptimisationTarget.MIN_COVER, **kw)
    cfg.optimisation_target = u.OptimisationTarget.ENERGY.value
    assert _lib.lib.eco_env_state_bytes(ctypes.byref(cfg), 4) == 0
