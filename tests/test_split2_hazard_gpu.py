"""The fp16x2 operand split of the dense kernels (split2_pk, eco_mpnn_dense2.h) emits v_fma_mix{lo,hi}_f16 as inline
asm with its own trailing wait states: the compiler's hazard recognizer cannot see inside asm, and an MFMA that
reads a VGPR written by VALU needs them (round 4: without them the paired and single forwards differed in the last
bits).  eco_probe_split2_mfma runs the split inside an MFMA chain as the dense kernels' mm_fh does (order 0), with
the lo fragment consumed first, straight after the asm (order 1), and -- the discriminating case -- with the split's
eight v_fma_mix and the first MFMA reading its lo fragment in ONE asm block built from the product's own asm text and
wait states (ECO_MIXLO / ECO_MIXHI / ECO_SPLIT2_WAIT), so the MFMA reads the register the last v_fma_mixhi wrote
with only those wait states between them (order 2; in orders 0 / 1 the compiler may place other instructions
there).  Each beside the same products from a plain-conversion split (cvt / subtract / cvt): the accumulators must
be bitwise equal for random activations, weights and scales.  The negative control -- the library built without the
wait states (ECO_SPLIT2_NEGATIVE_CONTROL, tools/r06/split2_negative.sh) -- must fail order 2; its log is
profiles/r06/split2_negative_control.log."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("order", [0, 1, 2])
def test_split2_asm_matches_plain_split_inside_mfma_chain(order):
    from eco_hip import _lib
    rng = np.random.default_rng(order)
    nb = 4096
    # activations over many binades (ReLU outputs, some zeros), per-block scales 2^k placing the block max near 2^14
    x = (rng.standard_normal((nb, 64, 16)) * np.exp2(rng.integers(-20, 10, (nb, 1, 1)))).astype(np.float32)
    x[rng.random(x.shape) < 0.2] = 0.0
    mx = np.abs(x).reshape(nb, -1).max(1)
    k = np.where(mx > 0, 15 - np.frexp(mx)[1], 0)
    sf = np.exp2(k).astype(np.float32)
    # weight fragments: random finite fp16 values (hi pieces) and small lo pieces
    w = np.concatenate([rng.standard_normal(8 * 512) * 1e4, rng.standard_normal(8 * 512) * 1e-1]).astype(np.float16)
    xt, st, wt = torch.from_numpy(x).cuda(), torch.from_numpy(sf).cuda(), torch.from_numpy(w.view(np.uint16)).cuda()
    out = torch.empty(2, nb, 16, 64, dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib.eco_probe_split2_mfma(_lib.ptr(xt), _lib.ptr(st), _lib.ptr(wt), nb, order, _lib.ptr(out),
                                             _lib.stream_ptr()))
    torch.cuda.synchronize()
    a, r = out[0].cpu().numpy(), out[1].cpu().numpy()
    assert np.isfinite(r).all() and np.abs(r).max() > 0
    bad = (a.view(np.uint32) != r.view(np.uint32))
    assert not bad.any(), f"{int(bad.sum())} of {bad.size} accumulators differ from the plain split"
