"""One line per bench JSON file: config, ms/step, roofline frac, phases."""
import json
import sys

for path in sys.argv[1:]:
    try:
        for line in open(path):
            line = line.strip()
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            cfg = d.get("config", {})
            print(path, cfg.get("config"), f"{d['ms_per_step']:.2f} ms", f"frac {d['roofline']['frac']:.4f}",
                  d.get("phases_ms"), d.get("cpu_baseline"))
    except (OSError, ValueError, KeyError) as e:
        print(path, "unreadable:", e)
