"""Board power and shader clock of this rank's GPU while a benchmark runs (sysfs, read-only).

MI355X boards hold their power cap through a training step (~1.3-1.4 kW) and trade shader clock for it: the
library GEMMs of the Llama-3-8B step ran at ~1.9 GHz of the 2.4 GHz maximum (``profiles/r4_gemm_roofline.md``), and
boxes of the pool differ by a few percent in the clock they hold -- the same code measures a few percent apart on
two boxes. ``bench.py`` samples both every 0.5 s over the timed steps and reports them next to the tokens/s, so a
number can be read against the clock it was measured at (sampling every 0.1 s cost the Llama-3-8B step ~0.25 %,
``profiles/r6_bench_telemetry_ab.jsonl``).

Sources: ``/sys/bus/pci/devices/<gpu>/hwmon/hwmon*/power1_average`` (µW; ``power1_input`` where the average is
absent) and ``pp_dpm_sclk`` (the DPM level marked ``*`` is the current clock). Nothing is written.
"""
from __future__ import annotations

import glob
import statistics
import threading
import time


def parse_sclk(text: str) -> int | None:
    """Current shader clock (MHz) from ``pp_dpm_sclk`` text: the line marked with ``*``."""
    for line in text.splitlines():
        line = line.strip()
        if line.endswith("*"):
            try:
                v = line.split(":", 1)[1].strip().rstrip("*").strip()
                return int(v.lower().split("mhz")[0].strip())
            except (IndexError, ValueError):
                return None
    return None


def summarize(values: list) -> dict | None:
    xs = [v for v in values if v is not None]
    if not xs:
        return None
    return {"n": len(xs), "mean": round(statistics.mean(xs), 1), "min": round(min(xs), 1), "max": round(max(xs), 1)}


def gpu_sysfs_dirs(device_index: int) -> tuple[str, str | None] | None:
    """(PCI device dir, hwmon dir or None) of a visible GPU, or None when sysfs does not show it."""
    try:
        from ..parallel.dist import _gpu_pci_dir

        d = _gpu_pci_dir(device_index)
    except Exception:  # noqa: BLE001 -- no GPU, no properties, no sysfs: telemetry is optional
        return None
    hw = sorted(glob.glob(d + "/hwmon/hwmon*"))
    return d, (hw[0] if hw else None)


class PowerClockSampler:
    """Samples (time, board power W, shader clock MHz) every ``period`` s on a daemon thread."""

    def __init__(self, device_index: int = 0, period: float = 0.1, where=None):
        self.period = period
        self.where = where if where is not None else gpu_sysfs_dirs(device_index)
        self.samples: list = []
        self._stop = threading.Event()
        self._t = None

    def read(self):
        if not self.where:
            return None
        dev, hw = self.where
        p = c = None
        if hw:
            for f in ("power1_average", "power1_input"):
                try:
                    with open(f"{hw}/{f}") as fh:
                        p = int(fh.read()) / 1e6
                    break
                except (OSError, ValueError):
                    continue
        try:
            with open(f"{dev}/pp_dpm_sclk") as fh:
                c = parse_sclk(fh.read())
        except OSError:
            pass
        return (time.time(), p, c)

    def _loop(self):
        while not self._stop.is_set():
            r = self.read()
            if r is not None:
                self.samples.append(r)
            self._stop.wait(self.period)

    def start(self) -> "PowerClockSampler":
        self.samples, self._stop = [], threading.Event()
        if self.where:
            self._t = threading.Thread(target=self._loop, name="kop-gpu-telemetry", daemon=True)
            self._t.start()
        return self

    def stop(self) -> dict | None:
        """Stop sampling; {"power_w": {n, mean, min, max}, "sclk_mhz": {...}} or None without sysfs access."""
        self._stop.set()
        if self._t is not None:
            self._t.join()
            self._t = None
        if not self.where:
            return None
        return {"power_w": summarize([s[1] for s in self.samples]),
                "sclk_mhz": summarize([s[2] for s in self.samples]),
                "period_s": self.period}
