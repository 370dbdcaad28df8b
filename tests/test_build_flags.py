"""The product library is built in one form only: the sources carry no build-time
A/B or probe macro a -D could flip, and the Makefile passes no -D beyond the platform define gcc
needs to read the HIP runtime headers. Measured-and-dropped forms live in DESIGN.md and git history;
tools/ab_libs.sh builds its variants from patched copies outside the product tree."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "shadow_amd", "csrc")
ALLOWED_D = {"__HIP_PLATFORM_AMD__"}
# include guards and the device-only switch of fw16.hip (tools/fwh_variants.hip includes the
# kernels without the host code); neither changes a result
ALLOWED_IFNDEF = {"SRT_FW16_DEVICE_ONLY"}


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".c", ".h")):
            with open(os.path.join(CSRC, f)) as fh:
                yield f, fh.read()


def test_makefile_defines_nothing_but_the_platform():
    with open(os.path.join(CSRC, "Makefile")) as f:
        mk = f.read()
    defs = set(re.findall(r"-D\s*([A-Za-z_][A-Za-z0-9_]*)", mk))
    assert defs <= ALLOWED_D, defs - ALLOWED_D
    assert not os.environ.get("EXTRA"), "EXTRA would add flags to the product build"


def test_no_overridable_macros_in_product_sources():
    bad = []
    for f, s in _sources():
        for m in re.finditer(r"^\s*#\s*ifndef\s+([A-Za-z_][A-Za-z0-9_]*)\s*\n\s*#\s*define\s+\1\b(.*)$",
                             s, re.M):
            name, rest = m.group(1), m.group(2).strip()
            guard = rest == "" and name.endswith("_H")
            if not guard and name not in ALLOWED_IFNDEF:
                bad.append(f"{f}: {name}")
        for m in re.finditer(r"^\s*#\s*(?:if|elif)\s+(?!defined)([A-Z][A-Z0-9_]+)\b", s, re.M):
            if m.group(1) not in ALLOWED_IFNDEF:
                bad.append(f"{f}: #if {m.group(1)}")
    assert not bad, bad
