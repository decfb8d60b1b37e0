#!/usr/bin/env python3
"""Fill the round-5 protocol table and hypothesis line of BASELINE.md from profiles/protocol_r5/ (table.md and
analysis/summary.json, written by tools/collect_protocol.sh); re-run after every re-collection."""
import json
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
b = (ROOT / "BASELINE.md").read_text()
table = (ROOT / "profiles/protocol_r5/table.md").read_text().strip()
hyp = json.loads((ROOT / "profiles/protocol_r5/analysis/summary.json").read_text())["hypotheses"]
line = ", ".join(f"{k} {'supported' if v.get('supported') else 'not supported'}" for k, v in sorted(hyp.items()))
start = b.index("### Protocol, round 5")
end = b.index("Deployment time (launcher start", start)
sec = b[start:end]
sec = re.sub(r"(\n\| arm \| users \|.*?\n)(?=\n)", "\n", sec, flags=re.S) if "| arm | users |" in sec else sec
sec = sec.replace("PROTOCOL_TABLE_R5", table) if "PROTOCOL_TABLE_R5" in sec else sec.rstrip() + "\n\n" + table + "\n\n"
b = b[:start] + sec + b[end:]
b = re.sub(r"Hypotheses on this engine \(`profiles/protocol_r5/analysis/summary.md`\): .*\n",
           f"Hypotheses on this engine (`profiles/protocol_r5/analysis/summary.md`): {line}.\n", b)
b = b.replace("HYPOTHESES_R5", line + ".")
(ROOT / "BASELINE.md").write_text(b)
print(line)
