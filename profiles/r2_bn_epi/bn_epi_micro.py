#!/usr/bin/env python
"""BatchNorm-statistics dgrad epilogue vs the BN's separate reduction pass, per ResNet-18 layer (B = 64).

For every conv stage whose dgrad stores a BatchNorm output's final gradient (``_Gemm.bn_epi_for`` of the
layer-wise plan): the plain dgrad, the dgrad with the BN-statistics epilogue (``conv_dgrad(bn_epi=...)``),
the full two-pass BN backward and its apply pass alone (``pre_reduced``), each replayed in a hipGraph.
fused = dgrad+epi + apply; unfused = dgrad + full BN backward.
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))
import torch  # noqa: E402

from micro import graph_time  # noqa: E402


def main():
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.train import layerwise as LW
    torch.cuda.set_device(0)
    tde.backend.set_random_seed(0)
    m = tde.zoo.resnet18()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1))
    B = int(os.environ.get("BATCH", "64"))
    prog = m._program("train", B)
    plan = prog.plans[0]
    x = torch.rand((1, B, 224, 224, 3)).cuda()
    y = torch.randint(0, 1000, (1, B)).to(torch.int32).cuda()
    prog.stage([(x, y)])
    prog.run()
    torch.cuda.synchronize()
    tot = dict(d=0.0, de=0.0, bn=0.0, ap=0.0)
    for st in plan.stages:
        if not (isinstance(st, LW._Gemm) and st.bn_epi_for is not None):
            continue
        bn = st.bn_epi_for
        g = st.geo.with_batch(B)
        dout = st.out.root().grad
        dx = st.inp.root().grad
        acc = st.accum[st.inp.root().id]
        R, C = bn.inp.rows(B), bn.inp.C
        ir = bn.inp.root()
        rr = bn.res.root() if bn.res is not None else None
        dxb = torch.empty_like(ir.grad)
        dres = torch.empty_like(rr.grad) if rr is not None else None

        def bwd(pre):
            O.bn_bwd(dx, ir.buf, R, C, mode=1, saved=bn.saved, gamma=bn.gamma, beta=bn.beta,
                     res=rr.buf if rr is not None else None, relu=bn.relu, dstats=bn.dstats, dx=dxb, dres=dres,
                     dgamma=bn.ggamma, dbeta=bn.gbeta, pre_reduced=pre)

        t_d = graph_time(lambda: O.conv_dgrad(dout, st.Wrow, dx, g, accum=acc, scratch=plan.scratch), 20)
        taken = []
        t_de = graph_time(lambda: taken.append(O.conv_dgrad(dout, st.Wrow, dx, g, accum=acc, scratch=plan.scratch,
                                                            bn_epi=bn.epi_args())), 20)
        t_bn = graph_time(lambda: bwd(False), 20)
        t_ap = graph_time(lambda: bwd(True), 20)
        for k, v in zip("d de bn ap".split(), (t_d, t_de, t_bn, t_ap)):
            tot[k] += v
        print(f"{st.layer.name:<22} {g.H}x{g.W}x{g.C}<-{g.Co} k{g.KH}s{g.sh} res={rr is not None:d} taken={taken[-1]:d} "
              f"| dgrad {t_d:6.1f} +epi {t_de:6.1f} | bn bwd {t_bn:6.1f} apply {t_ap:6.1f} | unfused "
              f"{t_d + t_bn:6.1f} fused {t_de + t_ap:6.1f} us", flush=True)
    print(f"TOTAL dgrad {tot['d']:.1f} +epi {tot['de']:.1f} | bn bwd {tot['bn']:.1f} apply {tot['ap']:.1f} | "
          f"unfused {tot['d'] + tot['bn']:.1f} fused {tot['de'] + tot['ap']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
