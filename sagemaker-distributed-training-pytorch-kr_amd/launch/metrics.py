"""Regex metric scraping over job stdout.

The notebooks define ``metric_definitions=[{'Name': ..., 'Regex': ...}]`` (NB1:301-307,
NB2:425-436) that SageMaker applies to the job log. ``MetricScraper`` applies the same
definitions line by line and keeps a time series per metric; the job writes them to
``metrics.json``. NOTE (reference bug kept visible, not silently fixed): NB1's
``'Train Loss: (.*?),'`` never matches the MNIST script's ``Loss: x`` line.
"""
from __future__ import annotations

import json
import re
import time
from typing import Dict, List, Optional


class MetricScraper:
    def __init__(self, metric_definitions: Optional[List[Dict[str, str]]] = None):
        self.defs = []
        for d in metric_definitions or []:
            self.defs.append((d["Name"], re.compile(d["Regex"])))
        self.series: Dict[str, List[dict]] = {n: [] for n, _ in self.defs}

    def feed(self, line: str):
        for name, rx in self.defs:
            m = rx.search(line)
            if m and m.groups():
                try:
                    v = float(m.group(1))
                except ValueError:
                    continue
                self.series[name].append({"timestamp": time.time(), "value": v})

    def last(self, name):
        s = self.series.get(name) or []
        return s[-1]["value"] if s else None

    def dump(self, path: str):
        with open(path, "w") as f:
            json.dump(self.series, f, indent=1)
