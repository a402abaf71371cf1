"""The ctypes mirrors of the kernels' argument structs (ops/kernels.py) have the size of the C++ structs
they stand for (csrc/include/tde_convnet.h, tde_optim.h, csrc/comm/xgmi_allreduce.hip).  A field added on
one side only would shift every later field of a struct passed by pointer: read without a GPU, from the
built library's host-side size exports."""
import ctypes as C

import pytest

from tensorflow_distributed_example_amd import _native as N


def _sizes(fn, n):
    out = (C.c_longlong * n)()
    got = fn(out, n)
    assert got == n
    return list(out)


@pytest.mark.skipif(not N.hip_available(), reason="libtde_hip.so not built")
def test_fused_step_structs_match_the_kernels():
    from tensorflow_distributed_example_amd.ops import kernels as K
    step, bwd, flat, hyper = _sizes(N.hip().tde_cnet_abi_sizes, 4)
    assert C.sizeof(K.StepOpt) == step
    assert C.sizeof(K.BwdOpt) == bwd
    assert C.sizeof(K.FlatApply) == flat
    assert C.sizeof(K.OptHyper) == hyper


@pytest.mark.skipif(not N.hip_available(), reason="libtde_hip.so not built")
def test_xgmi_structs_match_the_kernels():
    from tensorflow_distributed_example_amd.ops import kernels as K
    apply_, push = _sizes(N.hip().tde_xgmi_abi_sizes, 2)
    assert C.sizeof(K.XgApply) == apply_
    assert C.sizeof(K.XgPush) == push
