"""Iteration logger -- same API as the reference SCvx/utils/logging.py:6-52 (records list, log,
save_csv, save_json, clear)."""
import csv
import json
from typing import Dict, List


class Logger:
    def __init__(self):
        self.records: List[Dict] = []

    def log(self, record: Dict) -> None:
        self.records.append(record)

    def save_csv(self, filepath: str) -> None:
        if not self.records:
            return
        keys = list(self.records[0].keys())
        with open(filepath, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(self.records)

    def save_json(self, filepath: str) -> None:
        with open(filepath, "w") as f:
            json.dump(self.records, f, indent=2, default=float)

    def clear(self) -> None:
        self.records = []
