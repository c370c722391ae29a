"""Documentation stays in step with the code (CPU only):

* every environment switch librps reads (`env_int("RPS_...")` / `getenv("RPS_...")` in the HIP
  sources) has a row in INTEGRATION.md's switch table, so an A/B knob cannot ship undocumented;
* DESIGN.md's live sections (§0 to §10, before Appendix A) stay within 300 lines."""
import glob
import os
import re

from conftest import ROOT

CSRC = os.path.join(ROOT, "rust-particle-system_amd", "csrc")


def source_switches():
    names = set()
    for path in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp")):
        names.update(re.findall(r"(?:env_int|getenv)\(\s*\"(RPS_[A-Z0-9_]+)\"", open(path).read()))
    return names


def test_every_switch_documented():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    # "RPS_SPH_BATCH_D / _S" documents RPS_SPH_BATCH_S as a suffix of its row
    documented = set(re.findall(r"RPS_[A-Z0-9_]+", doc))
    for row in re.findall(r"`(RPS_[A-Z0-9_]+?)_[A-Z]+` / `_([A-Z]+)`", doc):
        documented.add(f"{row[0]}_{row[1]}")
    names = source_switches()
    assert names, "no switches found: the pattern no longer matches the sources"
    missing = sorted(n for n in names if n not in documented)
    assert not missing, f"switches read by librps but absent from INTEGRATION.md: {missing}"


def test_design_live_sections_length():
    lines = open(os.path.join(ROOT, "DESIGN.md")).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("## 0."))
    end = next(i for i, l in enumerate(lines) if l.startswith("## Appendix A"))
    assert end - start <= 300, f"DESIGN.md §0-§10 is {end - start} lines (limit 300)"
