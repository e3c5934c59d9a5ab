"""Network-adjusted time (src/timedata.cpp).

AddTimeData: every peer's version timestamp minus our clock is a sample (one per address, at
most 200 kept); once at least 5 samples are held and their count is odd, the median becomes the
node's time offset if it is within -maxtimeadjustment (default 70 minutes), else the offset is
reset to 0 and, if no peer agrees with our clock within 5 minutes, a warning is logged once
("Please check that your computer's date and time are correct!").
"""
from __future__ import annotations

import threading

from ..utils import log

DEFAULT_MAX_TIME_ADJUSTMENT = 70 * 60
MAX_SAMPLES = 200


class TimeData:
    def __init__(self, max_adjustment: int = DEFAULT_MAX_TIME_ADJUSTMENT):
        self.max_adjustment = max_adjustment
        self.offset = 0
        self._seen: set[str] = set()
        self._samples: list[int] = [0]  # CMedianFilter starts with our own 0 offset
        self._warned = False
        self._lock = threading.Lock()

    def add(self, ip: str, offset: int) -> int:
        """Record peer `ip`'s clock offset in seconds; returns the node's current offset."""
        with self._lock:
            if ip in self._seen or len(self._seen) >= MAX_SAMPLES:
                return self.offset
            self._seen.add(ip)
            self._samples.append(int(offset))
            if len(self._samples) > MAX_SAMPLES:
                self._samples.pop(0)
            n = len(self._samples)
            if n >= 5 and n % 2 == 1:
                median = sorted(self._samples)[n // 2]
                if abs(median) <= self.max_adjustment:
                    self.offset = median
                else:
                    self.offset = 0
                    if not self._warned and not any(0 < abs(s) <= 5 * 60 for s in self._samples):
                        self._warned = True
                        log.log_printf("Warning: Please check that your computer's date and time are correct! "
                                       "If your clock is wrong, Clore will not work properly.")
                log.log_print("net", f"time offset {self.offset:+d}s from {n} samples")
            return self.offset
