"""Occupancy guard for the hot kernels (CPU test: reads the gfx950 code objects inside
librpamd.so, no device needed).

Round 5 lost 15 % of the 2^22 fold to an A/B knob that raised k_bk_scatter to 94 VGPRs (one
1,024-thread tile per CU instead of two) without any test noticing (`profiles/LOG.md`, round 5
item 3). The designs in DESIGN.md §4 assume the workgroups per CU pinned below; the code
object's own metadata (`.vgpr_count`, `.agpr_count`, `.group_segment_fixed_size`,
`.max_flat_workgroup_size`) says what the hardware will give.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
LDS_PER_CU = 160 * 1024
SIMDS = 4

# kernel (a substring of the mangled name) -> workgroups per CU the design relies on
EXPECT = {
    # the bucket fold: two scatter tiles and three fold workgroups a CU
    "k_bk_scatterILb0E": 2,
    "k_bk_foldILb1E": 3,
    # the C2 lookupN(3) kernel: 4 workgroups (16 waves) a CU
    "k_lookupn_leanILi8ELi3ELi4ELb0ELi0ELi1E": 4,
    # the C5 refresh: two 4-wave workgroups a CU, two chain waves a SIMD
    "10k_ck_lanesE": 2,
}
# (every kernel named here carries __launch_bounds__ equal to its launch size, so the metadata's
# .max_flat_workgroup_size is the workgroup the launcher uses)


def _kernels(lib):
    """{mangled name: {field: int}} from the gfx950 code objects' metadata notes."""
    tmp = tempfile.mkdtemp()
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(lib, so)  # llvm-objdump --offloading writes the bundles beside its input
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], check=True,
                       capture_output=True, cwd=tmp)
        out = {}
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(tmp, f)],
                                   check=True, capture_output=True, text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"^(  - |    )\.(\w+):\s+(\S+)", line)
                if not m:
                    continue
                if m.group(1) == "  - ":
                    cur = {}
                if cur is None:
                    continue
                key, val = m.group(2), m.group(3)
                if key == "name":
                    out[val] = cur
                elif val.isdigit():
                    cur[key] = int(val)
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _per_cu(k):
    """Workgroups per CU: the least of the VGPR, LDS and wave-slot limits (MI355X_MICROARCH.md:
    one 512-entry register file per SIMD lane, allocated in granules of 8; 8 waves per SIMD)."""
    regs = k.get("vgpr_count", 0) + k.get("agpr_count", 0)
    alloc = max(8, (regs + 7) // 8 * 8)
    waves_simd = min(8, 512 // alloc)
    wg_waves = (k["max_flat_workgroup_size"] + 63) // 64
    per_simd = (wg_waves + SIMDS - 1) // SIMDS
    by_regs = waves_simd // per_simd
    lds = k.get("group_segment_fixed_size", 0)
    by_lds = LDS_PER_CU // lds if lds else 1 << 30
    return min(by_regs, by_lds, 32 // wg_waves)


@pytest.fixture(scope="module")
def kernels(rpa):
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("no ROCm LLVM tools")
    return _kernels(rpa.LIB_PATH)


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_hot_kernel_occupancy(kernels, name):
    hits = {n: k for n, k in kernels.items() if name in n}
    assert hits, f"{name}: no such kernel in the library"
    for n, k in hits.items():
        got = _per_cu(k)
        assert got >= EXPECT[name], (f"{n}: {got} workgroups a CU (VGPRs {k.get('vgpr_count')}, "
                                     f"LDS {k.get('group_segment_fixed_size')} B), the design assumes "
                                     f"{EXPECT[name]}")
