"""Code-object checks of the gfx950 kernels (CPU: reads the offload bundle metadata of the in-tree build).

The xGMI all-reduce kernels spin on flags raised by other workgroups (of the same grid, of the other
replicas' grids, of other processes): they rely on every workgroup of the grid being resident at once.
A kernel that needs scratch (private segment) memory is dispatched only as far as the queue's scratch
allocation reaches, which can leave some of its workgroups waiting for others that spin forever — so the
waiting kernels must use no scratch at all (register-resident state only)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(obj, tmp_path):
    if not os.path.exists(obj) or not shutil.which(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("in-tree build objects / LLVM tools not available")
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], check=True,
                           stdout=subprocess.PIPE, text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_count|uses_dynamic_stack):\s+(\S+)", line)
        if not m:
            continue
        cur[m.group(1)] = m.group(2)
        if "name" in cur and "private_segment_fixed_size" in cur and "vgpr_count" in cur:
            out[cur.pop("name")] = dict(cur)
            cur = {}
    return out


def test_xgmi_allreduce_kernels_use_no_scratch(tmp_path):
    ks = _kernels(os.path.join(ROOT, "build", "obj", "xgmi_allreduce.hip.o"), tmp_path)
    xg = {k: v for k, v in ks.items() if "xgmi_allreduce_kernel" in k}
    assert len(xg) == 4, ks.keys()
    for name, meta in xg.items():
        assert meta["private_segment_fixed_size"] == "0", (name, meta)
        assert meta.get("uses_dynamic_stack", "false") == "false", (name, meta)
