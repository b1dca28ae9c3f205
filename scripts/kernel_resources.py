"""Register, LDS and spill counts of the engine library's kernels, from the
gfx950 code objects' AMDGPU metadata (llvm-readelf --notes), e.g. to check
that a variant of k_fused still fits 4 waves per SIMD (<= 128 VGPRs).

  python scripts/kernel_resources.py [library.so] [name filter]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "topoflow-glacier_amd"))

from topoflow_glacier import _native as nat  # noqa: E402

lib = Path(sys.argv[1]) if len(sys.argv) > 1 else nat.LIB_PATH
flt = sys.argv[2] if len(sys.argv) > 2 else "k_fused"
readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
for i, elf in enumerate(nat.gfx950_code_objects(lib)):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf)
        f.flush()
        notes = subprocess.run([readelf, "--notes", f.name], capture_output=True, text=True).stdout
    for block in re.split(r"\n  - ", notes)[1:]:
        name = re.search(r"\n    \.name:\s+(\S+)", block)
        if not name or flt not in name.group(1):
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", block) or [None, "?"])[1]  # noqa: E731
        print(f"unit{i} {name.group(1)[:72]:72s} vgpr={get('vgpr_count')} sgpr={get('sgpr_count')} "
              f"vgpr_spill={get('vgpr_spill_count')} sgpr_spill={get('sgpr_spill_count')} "
              f"lds={get('group_segment_fixed_size')} scratch={get('private_segment_fixed_size')}")
