"""The dispatcher's defaults (oneccl_amd/csrc/comp.cpp kHostMax*Default,
kHostShare*Default) against what tools/dispatch_sweep.py --recommend derives
from the committed MI355X sweeps (profiles/round2_dispatch/): the thresholds
must be the measured crossovers and the default share within one sweep step
of the best measured split."""
from __future__ import annotations

import json
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _rows():
    merged = {}
    for name in ("dispatch_sweep.jsonl", "coop_sweep.jsonl"):
        for line in (ROOT / "profiles" / "round2_dispatch" / name).read_text().splitlines():
            if line.startswith("{"):
                r = json.loads(line)
                if r.get("dtype") == "f32":
                    merged.setdefault((r["kind"], r["bytes"]), {}).update(r)
    return list(merged.values())


def _default(name):
    src = (ROOT / "oneccl_amd" / "csrc" / "comp.cpp").read_text()
    m = re.search(rf"static const \w+ {name} = ([0-9.]+)(ull << (\d+))?;", src)
    return float(m.group(1)) * (2 ** int(m.group(3)) if m.group(3) else 1)


def test_defaults_match_the_measured_crossovers():
    import sys
    sys.path.insert(0, str(ROOT))
    from tools.dispatch_sweep import recommend
    rec = recommend(_rows())
    assert rec["pageable"]["host_max_bytes"] == _default("kHostMaxPageableDefault")
    assert rec["pinned"]["host_max_bytes"] == _default("kHostMaxPinnedDefault")
    assert abs(rec["pageable"]["share"] - _default("kHostShareDefault")) <= 0.1
    assert abs(rec["pinned"]["share"] - _default("kHostSharePinnedDefault")) <= 0.1
