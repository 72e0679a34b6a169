"""Per-kernel register / scratch / occupancy summary of libkalibr_hip (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/resource_usage.py [filter-substring] [extra hipcc flags...]
"""
import re
import subprocess
import sys

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
from kalibr_amd import build as B  # noqa: E402

flt = sys.argv[1] if len(sys.argv) > 1 else ""
extra = sys.argv[2:]
r = subprocess.run([B.HIPCC] + B.FLAGS + extra + ["-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/tmp/ru.o", B.SRC],
                   capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
keys = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]"]
for fn, kv in rows.items():
    dem = subprocess.run(["c++filt", fn], capture_output=True, text=True).stdout.strip()
    if flt in dem:
        print(f"{dem[:60]:60s} " + " ".join(f"{k.split(' [')[0].replace(' ', '_')}={kv.get(k, '-')}" for k in keys))
