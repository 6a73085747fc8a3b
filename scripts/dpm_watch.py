"""Read-only sampler of the GPU's DPM clock levels (sysfs pp_dpm_{sclk,mclk,
fclk,socclk}: the level marked '*' is the current one) on a thread, for
diagnostics: does the memory or fabric clock drop while the GPU runs PCIe
copies or idles, and stay low for the next kernel?  Nothing is written."""
import ctypes as C
import os
import threading
import time

CLOCKS = ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk")


def sysfs_dir(device=0):
    hip = C.CDLL("libamdhip64.so")
    buf = C.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
        return None
    bdf = buf.value.decode().lower()
    d = f"/sys/bus/pci/devices/{bdf}"
    return d if os.path.isdir(d) else None


def current(path):
    try:
        with open(path) as fh:
            for ln in fh:
                if ln.rstrip().endswith("*"):
                    return ln.split(":", 1)[1].strip().rstrip("*").strip()
    except OSError:
        return None
    return None


class Watch:
    def __init__(self, device=0, period_s=0.0005):
        self.dir = sysfs_dir(device)
        self.files = [c for c in CLOCKS if self.dir and os.path.exists(os.path.join(self.dir, c))]
        self.period = period_s
        self.samples = []          # (t, label, {clock: level})
        self.label = "start"
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            t = time.perf_counter()
            self.samples.append((t, self.label, {c: current(os.path.join(self.dir, c)) for c in self.files}))
            time.sleep(self.period)

    def start(self):
        if self.files:
            self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join()

    def report(self):
        """Per label: how often each clock sat at each level, and samples taken."""
        out = {}
        for _, lab, lv in self.samples:
            d = out.setdefault(lab, {"samples": 0})
            d["samples"] += 1
            for c, v in lv.items():
                d.setdefault(c, {}).setdefault(v, 0)
                d[c][v] += 1
        return {"sysfs": self.dir, "clocks": self.files, "by_phase": out}
