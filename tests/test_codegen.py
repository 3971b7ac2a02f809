"""Static check of the built gfx950 code objects (no GPU needed).

tools/vmcnt_scan.py flags partial `s_waitcnt vmcnt(k)` waits that retire a VMEM op issued
under one EXEC mask while an op issued under another stays outstanding: the shape that
returned stale registers under concurrent GPU load in the suffix sorter's key kernel
("Concurrent encodes"). Product kernels must have none.
"""
import glob
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _disassemble(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fat")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}",
                    "--unbundle"], check=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True)
    s = os.path.join(tmp, os.path.basename(obj) + ".s")
    open(s, "w").write(out.stdout)
    return s


@pytest.mark.skipif(not shutil.which(f"{LLVM}/llvm-objdump"), reason="ROCm LLVM tools absent")
def test_no_mixed_exec_partial_vmcnt(tmp_path):
    from vmcnt_scan import scan

    objs = sorted(glob.glob(os.path.join(ROOT, "salz_amd", "build", "*.o")))
    objs = [o for o in objs if not o.endswith("salz_host.o")]
    if not objs:
        pytest.skip("library not built (python -c 'import __graft_entry__ as g; g.build()')")
    hits = []
    for o in objs:
        hits += scan(_disassemble(o, str(tmp_path)))
    assert hits == [], hits


def test_scanner_flags_the_known_hazard(tmp_path):
    """The scanner's model on hand-written snippets: the k_sa_init shape (a load, then a load
    under a narrower EXEC mask, then a partial wait) is flagged; loads issued under one mask,
    or inside a completed if/else, are not."""
    from vmcnt_scan import scan

    bad = """0000000000000000 <k_bad>:
	global_load_dwordx2 v[4:5], v0, s[10:11]
	s_and_saveexec_b64 s[0:1], vcc
	s_cbranch_execz 13
	global_load_dwordx2 v[0:1], v[0:1], off offset:8
	s_waitcnt vmcnt(1)
	v_lshrrev_b64 v[4:5], v7, v[4:5]
	s_or_b64 exec, exec, s[0:1]
"""
    good = """0000000000000100 <k_good>:
	global_load_dwordx4 v[2:5], v2, s[2:3]
	s_and_saveexec_b64 s[0:1], vcc
	s_xor_b64 s[0:1], exec, s[0:1]
	v_mov_b32 v9, 0
	s_or_saveexec_b64 s[0:1], s[0:1]
	s_xor_b64 exec, exec, s[0:1]
	v_mov_b32 v9, 1
	s_or_b64 exec, exec, s[0:1]
	global_load_dwordx2 v[6:7], v[8:9], off
	s_waitcnt vmcnt(1)
"""
    # a loop latch laid out after an unconditional jump: its EXEC join is not a region change
    # for the loads linearly above it
    jump = """0000000000000200 <k_jump>:
	s_and_saveexec_b64 s[30:31], vcc
	global_load_dword v1, v[2:3], off
	global_load_dword v4, v[2:3], off offset:4
	s_branch 12
	s_or_b64 exec, exec, s[2:3]
	global_load_dword v5, v[6:7], off
	s_waitcnt vmcnt(1)
"""
    p = tmp_path / "snip.s"
    p.write_text(bad + good + jump)
    hits = scan(str(p))
    assert [k for k, _ in hits] == ["k_bad"], hits
