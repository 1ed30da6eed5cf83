"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel
(VGPRs, VGPR spills, SGPR spills, scratch).  usage: make resources 2>&1 | python3 tools/resources.py [filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    for key in ("VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "AGPRs"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m and cur is not None and key not in cur:
            cur[key] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>3} vspill {r.get('SGPRs Spill', '?'):>4} sspill "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>5} scratch  {r['name'][:110]}")
