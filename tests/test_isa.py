"""Machine-code checks of the built gfx950 code object (no GPU needed).

The tick kernels publish each result with a sequence number written after an L2 write-back
(``buffer_wbl2``, the release fence of ``publish_system`` / ``publish_agent`` in
``csrc/qmx_hip.hip``).  The write-back is itself a vector memory operation: the store that
publishes must wait for it (``s_waitcnt vmcnt(0)``), or the host can see the new sequence
number before the output bytes reach memory.  The compiler's waitcnt pass once dropped that
wait (a flag load had been waited just before, and the pass does not count the write-back):
the headline bench then returned 1-7 deltas per 2.6M responses from the previous tick's
output.  This test disassembles the in-tree extension and fails on any write-back that is
not waited for before the next store or control transfer.
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")
TOOLS = [LLVM / "llvm-objcopy", LLVM / "clang-offload-bundler", LLVM / "llvm-objdump", LLVM / "llvm-readelf"]


def _extension():
    sos = sorted((REPO / "quorum_amd").glob("_qmx*.so"))
    return sos[0] if sos else None


@pytest.fixture(scope="module")
def code_object(tmp_path_factory):
    """The in-tree extension's gfx950 code object (path)."""
    so = _extension()
    if so is None or not all(t.exists() for t in TOOLS):
        pytest.skip("extension not built or LLVM tools missing")
    d = tmp_path_factory.mktemp("isa")
    fat, co = d / "fat.bin", d / "dev.co"
    subprocess.run([str(TOOLS[0]), f"--dump-section=.hip_fatbin={fat}", str(so), str(d / "host.so")],
                   check=True, capture_output=True)
    targets = subprocess.run([str(TOOLS[1]), "--list", "--type=o", f"--input={fat}"], check=True,
                             capture_output=True, text=True).stdout.split()
    gfx = [t for t in targets if t.endswith("gfx950")]
    assert gfx, f"no gfx950 code object in {so.name}: {targets}"
    subprocess.run([str(TOOLS[1]), "--unbundle", "--type=o", f"--input={fat}", f"--targets={gfx[0]}",
                    f"--output={co}"], check=True, capture_output=True)
    return co


@pytest.fixture(scope="module")
def disasm(code_object):
    out = subprocess.run([str(TOOLS[2]), "-d", "--no-show-raw-insn", str(code_object)], check=True,
                         capture_output=True, text=True).stdout
    return out.splitlines()


def kernel_resources(notes: str):
    """{kernel symbol: {field: int}} from `llvm-readelf --notes` (the AMDHSA metadata: one YAML
    map per kernel, a `- ` item each, its keys sorted — some before `.name`)."""
    out, cur = [], None
    for line in notes.splitlines():
        if re.match(r"\s*-\s+\.", line):  # a new kernel's map begins
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
        if m:
            cur["name"] = m.group(1)
            continue
        m = re.match(r"\s*-?\s*\.(private_segment_fixed_size|vgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"group_segment_fixed_size):\s+(\d+)", line)
        if m:
            cur[m.group(1)] = int(m.group(2))
    return {d["name"]: d for d in out if "name" in d}


def _tick_kernels(code_object):
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(code_object)], check=True,
                           capture_output=True, text=True).stdout
    res = kernel_resources(notes)
    return {k: v for k, v in res.items() if "qmx_tick_kernel" in k or "qmx_tick_persistent" in k}


def test_tick_kernels_have_no_scratch(code_object):
    """The production tick kernels (one-shot, and the persistent grid's default variant with
    one workgroup per CU) keep everything in registers and LDS: no VGPR spills and no scratch
    beyond one saved register of a call — a spill to scratch is HBM traffic on every item's critical path.
    (SGPR spills go to VGPR lanes, not memory.)  The register-capped two-workgroups-per-CU
    variant (qmx_tick_persistent<4>, QMX_GRID_OCC=2) is allowed its measured scratch."""
    ticks = _tick_kernels(code_object)
    assert len(ticks) == 3, sorted(ticks)
    for name, r in ticks.items():
        assert r.get("group_segment_fixed_size", 0) <= 160 * 1024, (name, r)  # one CU's LDS
        if "ILi4E" in name:  # two per CU: 2 x LDS must fit one CU, at most 128 VGPRs
            assert 2 * r["group_segment_fixed_size"] <= 160 * 1024, (name, r)
            assert r["vgpr_count"] <= 128 and r.get("private_segment_fixed_size", 0) <= 512, (name, r)
            continue
        # (at most one callee-saved VGPR of the non-inlined s4_wave call is saved to the stack
        # at its entry and restored at its exit: 8 B, no spill inside any stage)
        assert r.get("private_segment_fixed_size") <= 16, (name, r)
        assert r.get("vgpr_spill_count", 0) == 0, (name, r)


def test_tick_kernel_register_ceilings(code_object):
    """Register use of the tick kernels may not creep up unnoticed (round-5 review: the
    persistent kernel's SGPR spills went 367 -> 377 with no test to say so).  Ceilings a little
    above the round-6 build: one-shot 171 VGPRs / 247 SGPR spills, persistent 256 / 364."""
    ticks = _tick_kernels(code_object)
    for name, r in ticks.items():
        if "qmx_tick_kernel" in name:
            assert r["vgpr_count"] <= 184 and r.get("sgpr_spill_count", 0) <= 270, (name, r)
        elif "ILi2E" in name:
            assert r["vgpr_count"] <= 256 and r.get("sgpr_spill_count", 0) <= 400, (name, r)
        else:
            assert r.get("sgpr_spill_count", 0) <= 400, (name, r)


_STORE = re.compile(r"^\s*(global_store|flat_store|buffer_store|global_atomic|flat_atomic|buffer_atomic)")
_LEAVE = re.compile(r"^\s*(s_branch|s_cbranch|s_setpc|s_endpgm|s_swappc)")
_WAIT = re.compile(r"^\s*s_waitcnt\b.*\bvmcnt\(0\)")


def unwaited_writebacks(lines):
    """(line, what) for every buffer_wbl2 reaching a store or a control transfer before an
    s_waitcnt vmcnt(0)."""
    bad = []
    for i, l in enumerate(lines):
        if "buffer_wbl2" not in l:
            continue
        for j in range(i + 1, min(i + 64, len(lines))):
            m = lines[j]
            if _WAIT.match(m):
                break
            if _STORE.match(m) or _LEAVE.match(m):
                bad.append((i + 1, m.strip().split("//")[0].strip()))
                break
    return bad


def test_unwaited_writeback_detector():
    ok = ["\tbuffer_wbl2 sc0 sc1", "\ts_waitcnt vmcnt(0)", "\tglobal_store_dword v1, v2, s[0:1] sc0 sc1"]
    bad = ["\tbuffer_wbl2 sc0 sc1", "\tglobal_store_dword v43, v217, s[0:1] offset:16 sc0 sc1"]
    assert unwaited_writebacks(ok) == []
    assert unwaited_writebacks(bad) == [(1, "global_store_dword v43, v217, s[0:1] offset:16 sc0 sc1")]


def test_every_l2_writeback_is_waited_before_publishing(disasm):
    n = sum("buffer_wbl2" in l for l in disasm)
    assert n >= 4, "expected the tick / finalize / relay publishes in the code object"
    assert unwaited_writebacks(disasm) == []
