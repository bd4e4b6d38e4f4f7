"""The built library's gfx950 code holds no 12/16-byte store with an SGPR soffset and no
wide store whose data registers the next VALU overwrites (the cause of round 5's r5m wrong
x / memory stores in the sign receive; tools/isa_hazards.py).  CPU only:
it disassembles the shipped code objects."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "chocosgd_amd", "lib", "libchoco_codec.so")

import isa_hazards  # noqa: E402


def test_scanner_flags_the_r5m_pattern():
    """The pattern the r5m build compiled to (a 16-B nt store with an SGPR soffset, then a
    packed add into its first data registers) is flagged; the same store followed by an
    unrelated VALU is counted but not flagged."""
    bad = ("\tbuffer_store_dwordx4 v[82:85], v1, s[36:39], s8 offen nt\n"
           "\tv_pk_add_f32 v[82:83], v[90:91], v[82:83] neg_lo:[0,1] neg_hi:[0,1]\n")
    ok = ("\tbuffer_store_dwordx4 v[82:85], v1, s[36:39], 0 offen nt\n"
          "\tv_and_b32_e32 v5, 32, v3\n")
    assert isa_hazards.scan_text(bad) == (1, 1, [(bad.splitlines()[0].strip(), bad.splitlines()[1].strip())])
    assert isa_hazards.scan_text(ok) == (1, 0, [])


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built (run __graft_entry__.build())")
def test_built_library_has_no_store_data_hazard():
    n_wide, n_sreg, bad = isa_hazards.scan_library(LIB)
    assert n_wide > 1000  # the scan saw the codec's kernels
    assert n_sreg == 0, "a 12/16-B buffer store takes an SGPR soffset"
    assert bad == [], bad[:5]
