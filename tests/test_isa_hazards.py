"""k_conv4_max's inline-asm screening keys read MFMA accumulators; hipcc does
not pad wait states inside an asm string, so the distance from the
accumulator's last MFMA comes from the schedule alone.
tools/check_asm_hazards.py compiles feat_fused.hip for gfx950 and checks every
such read against the 8-pass XDL requirement (12 wait states) along every
path, loop back edges included.  CPU only (hipcc cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "tools", "check_asm_hazards.py")

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")


def test_screening_asm_reads_are_past_the_mfma_hazard():
    r = subprocess.run([sys.executable, TOOL], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "below 12: 0" in r.stdout


def test_checker_flags_a_read_right_after_the_mfma(tmp_path):
    """The checker itself: a listing whose asm reads an accumulator two
    instructions after the MFMA that wrote it (and one where a loop back edge
    brings the MFMA close) must fail."""
    body = """_ZN5pcadv11k_conv4_maxILi3ELb0EEEvPKfiiS2_S2_PfPiPm:
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]
\tv_mov_b32 v30, 0
.LBB9_1:
\tv_add_u32 v31, v31, 1
\t;;#ASMSTART
\tv_ashrrev_i32 v40, 31, v3
\tv_bitop3_b32 v40, v3, v40, s4 bitop3:0x78
\t;;#ASMEND
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]
\ts_cbranch_scc1 .LBB9_1
\ts_endpgm
.Lfunc_end9:
"""
    p = tmp_path / "bad.s"
    p.write_text(body)
    r = subprocess.run([sys.executable, TOOL, "--asm", str(p)], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 1
    assert "below 12: 1" in r.stdout
