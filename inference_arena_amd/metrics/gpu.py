"""MI355X telemetry exporter (the GPU counterpart of the reference's cAdvisor
container CPU/memory series, infrastructure/prometheus/prometheus.yml:57-92).

Sources, first available wins:
  1. the ROCm ``amdsmi`` Python bindings (``/opt/rocm/share/amd_smi``),
  2. ``amd-smi metric --json`` / ``rocm-smi --json`` CLI,
  3. ``torch.cuda.mem_get_info`` (memory only).

Gauges (label ``gpu``): arena_gpu_utilization_percent,
arena_gpu_memory_used_bytes, arena_gpu_memory_total_bytes,
arena_gpu_power_watts, arena_gpu_temperature_celsius.

Run standalone: ``python -m inference_arena_amd.metrics.gpu --port 9400``.
"""
from __future__ import annotations

import json
import shutil
import subprocess
import sys
import threading
import time

from prometheus_client import CollectorRegistry, Gauge, generate_latest


def _try_amdsmi():
    try:
        if "/opt/rocm/share/amd_smi" not in sys.path:
            sys.path.append("/opt/rocm/share/amd_smi")
        import amdsmi  # type: ignore

        amdsmi.amdsmi_init()
        return amdsmi
    except Exception:  # noqa: BLE001 - optional dependency
        return None


class GpuTelemetry:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.util = Gauge("arena_gpu_utilization_percent", "GPU busy percent", ["gpu"], registry=r)
        self.mem = Gauge("arena_gpu_memory_used_bytes", "VRAM in use", ["gpu"], registry=r)
        self.mem_total = Gauge("arena_gpu_memory_total_bytes", "VRAM size", ["gpu"], registry=r)
        self.power = Gauge("arena_gpu_power_watts", "Socket power", ["gpu"], registry=r)
        self.temp = Gauge("arena_gpu_temperature_celsius", "Hotspot temperature", ["gpu"], registry=r)
        self.smi = _try_amdsmi()
        self.source = "amdsmi" if self.smi else ("cli" if shutil.which("amd-smi") else "torch")
        self._stop = threading.Event()

    def sample(self) -> list[dict]:
        rows = []
        if self.smi is not None:
            smi = self.smi
            for i, h in enumerate(smi.amdsmi_get_processor_handles()):
                row = {"gpu": str(i)}
                try:
                    row["util"] = float(smi.amdsmi_get_gpu_activity(h)["gfx_activity"])
                except Exception:  # noqa: BLE001
                    pass
                try:
                    v = smi.amdsmi_get_gpu_vram_usage(h)
                    row["mem"], row["mem_total"] = float(v["vram_used"]) * 2**20, float(v["vram_total"]) * 2**20
                except Exception:  # noqa: BLE001
                    pass
                try:
                    p = smi.amdsmi_get_power_info(h)
                    row["power"] = float(p.get("socket_power", p.get("current_socket_power", 0)))
                except Exception:  # noqa: BLE001
                    pass
                try:
                    row["temp"] = float(smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.HOTSPOT,
                                                                   smi.AmdSmiTemperatureMetric.CURRENT))
                except Exception:  # noqa: BLE001
                    pass
                rows.append(row)
            return rows
        if self.source == "cli":
            try:
                out = subprocess.run(["amd-smi", "metric", "--json"], capture_output=True, text=True, timeout=10)
                data = json.loads(out.stdout)
                for i, g in enumerate(data if isinstance(data, list) else data.get("gpu_data", [])):
                    row = {"gpu": str(g.get("gpu", i))}
                    try:
                        row["util"] = float(g["usage"]["gfx_activity"]["value"])
                    except (KeyError, TypeError, ValueError):
                        pass
                    try:
                        row["mem"] = float(g["mem_usage"]["used_vram"]["value"]) * 2**20
                        row["mem_total"] = float(g["mem_usage"]["total_vram"]["value"]) * 2**20
                    except (KeyError, TypeError, ValueError):
                        pass
                    try:
                        row["power"] = float(g["power"]["socket_power"]["value"])
                    except (KeyError, TypeError, ValueError):
                        pass
                    rows.append(row)
                return rows
            except (OSError, ValueError, subprocess.SubprocessError):
                pass
        try:
            import torch

            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                rows.append({"gpu": str(i), "mem": float(total - free), "mem_total": float(total)})
        except Exception:  # noqa: BLE001
            pass
        return rows

    def update(self) -> list[dict]:
        rows = self.sample()
        for r in rows:
            g = r["gpu"]
            for key, gauge in (("util", self.util), ("mem", self.mem), ("mem_total", self.mem_total),
                               ("power", self.power), ("temp", self.temp)):
                if key in r:
                    gauge.labels(g).set(r[key])
        return rows

    def start(self, interval_s: float = 1.0) -> threading.Thread:
        def loop():
            while not self._stop.is_set():
                self.update()
                self._stop.wait(interval_s)

        t = threading.Thread(target=loop, daemon=True, name="gpu-telemetry")
        t.start()
        return t

    def stop(self) -> None:
        self._stop.set()

    def render(self) -> bytes:
        return generate_latest(self.registry)


def main(argv=None) -> int:
    import argparse

    from prometheus_client import start_http_server

    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=9400)
    ap.add_argument("--interval", type=float, default=1.0)
    a = ap.parse_args(argv)
    t = GpuTelemetry()
    start_http_server(a.port, registry=t.registry)
    t.start(a.interval)
    print(f"GPU telemetry ({t.source}) on :{a.port}/metrics", flush=True)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    raise SystemExit(main())
