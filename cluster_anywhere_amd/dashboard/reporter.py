"""Per-node physical metrics: CPU, memory, disk, network, and per-GPU utilisation,
HBM, power and temperature (reference role:
``python/ray/dashboard/modules/reporter/reporter_agent.py:89-140``, GPU sampling
``:489``).

Every node samples itself -- the head node inside the head process, every other
node inside its node agent, which pushes the sample to the head (``node_stats``
message) -- every ``CAAMD_REPORTER_INTERVAL_S`` seconds (default 2; ``0``
disables). The head keeps the latest sample in its node table, so
``/api/v0/nodes`` carries it and ``/metrics`` exports it as the reference's
``ray_node_*`` Prometheus gauges.

GPUs are AMD Instinct only: through ``amdsmi`` (per-device GFX activity, VRAM
usage, socket power, hotspot temperature), falling back to the amdgpu sysfs files
(``gpu_busy_percent``, ``mem_info_vram_*``, hwmon ``power1_average`` /
``temp*_input``) when the library or its device access is unavailable. Nothing
here initialises HIP.
"""
from __future__ import annotations

import glob
import os
import socket
import threading
import time
from typing import Any, Callable, Dict, List, Optional

INTERVAL_S = float(os.environ.get("CAAMD_REPORTER_INTERVAL_S", "2.0"))


# ------------------------------------------------------------------ GPUs
class _AmdSmi:
    """amdsmi handles, opened once per process (None when unusable)."""

    def __init__(self):
        self.ok = False
        self.handles: List[Any] = []
        try:
            import amdsmi

            amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
            self.handles = list(amdsmi.amdsmi_get_processor_handles())
            self.mod = amdsmi
            self.ok = bool(self.handles)
        except Exception:
            self.ok = False

    def sample(self) -> List[Dict[str, Any]]:
        a = self.mod
        out = []
        for i, h in enumerate(self.handles):
            g: Dict[str, Any] = {"index": i}
            try:
                g["name"] = a.amdsmi_get_gpu_asic_info(h).get("market_name") or "AMD Instinct"
            except Exception:
                g["name"] = "AMD Instinct"
            try:
                g["pci_bus_id"] = str(a.amdsmi_get_gpu_device_bdf(h))
            except Exception:
                pass
            try:
                g["utilization_gpu"] = float(a.amdsmi_get_gpu_activity(h)["gfx_activity"])
            except Exception:
                g["utilization_gpu"] = None
            try:
                v = a.amdsmi_get_gpu_vram_usage(h)  # MiB
                g["memory_used"] = int(v["vram_used"]) << 20
                g["memory_total"] = int(v["vram_total"]) << 20
            except Exception:
                pass
            try:
                p = a.amdsmi_get_power_info(h)
                w = p.get("current_socket_power")
                if w in (None, "N/A", 0):
                    w = p.get("average_socket_power", p.get("socket_power"))
                g["power_w"] = float(w)
            except Exception:
                pass
            try:
                g["temperature_c"] = float(a.amdsmi_get_temp_metric(
                    h, a.AmdSmiTemperatureType.HOTSPOT, a.AmdSmiTemperatureMetric.CURRENT))
            except Exception:
                pass
            out.append(g)
        return out


_SMI: Optional[_AmdSmi] = None
_SMI_LOCK = threading.Lock()


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _sysfs_gpus() -> List[Dict[str, Any]]:
    out = []
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        if _read(os.path.join(dev, "vendor")) != "0x1002" or _read(os.path.join(dev, "gpu_busy_percent")) is None:
            continue
        g: Dict[str, Any] = {"index": len(out), "name": "AMD Instinct",
                             "pci_bus_id": os.path.basename(os.path.realpath(dev))}
        busy = _read(os.path.join(dev, "gpu_busy_percent"))
        g["utilization_gpu"] = float(busy) if busy and busy.isdigit() else None
        for k, key in (("mem_info_vram_used", "memory_used"), ("mem_info_vram_total", "memory_total")):
            v = _read(os.path.join(dev, k))
            if v and v.isdigit():
                g[key] = int(v)
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            p = _read(os.path.join(hw, "power1_average")) or _read(os.path.join(hw, "power1_input"))
            if p and p.isdigit():
                g["power_w"] = int(p) / 1e6
            temps = [_read(t) for t in sorted(glob.glob(os.path.join(hw, "temp*_input")))]
            temps = [int(t) / 1000.0 for t in temps if t and t.lstrip("-").isdigit()]
            if temps:
                g["temperature_c"] = max(temps)
        out.append(g)
    return out


def sample_gpus() -> List[Dict[str, Any]]:
    """One entry per AMD GPU on this node: index, name, pci_bus_id,
    utilization_gpu (%), memory_used / memory_total (bytes), power_w, temperature_c."""
    global _SMI
    if os.environ.get("CAAMD_REPORTER_GPU", "1") == "0":
        return []
    with _SMI_LOCK:
        if _SMI is None:
            _SMI = _AmdSmi()
        smi = _SMI
    if smi.ok:
        try:
            gpus = smi.sample()
            if gpus and any(g.get("utilization_gpu") is not None for g in gpus):
                return gpus
        except Exception:
            pass
    return _sysfs_gpus()


# ------------------------------------------------------------------ node
_prev_io: Dict[str, Any] = {}


def sample_node(session_dir: Optional[str] = None, gpus: Optional[Callable[[], List[Dict]]] = None) -> Dict[str, Any]:
    """CPU / memory / disk / network / GPU sample of this node (the reference's
    reporter fields, flattened)."""
    import psutil

    now = time.time()
    vm = psutil.virtual_memory()
    s: Dict[str, Any] = {
        "timestamp": now, "hostname": socket.gethostname(),
        "cpu_percent": float(psutil.cpu_percent(interval=None)),
        "cpu_count": psutil.cpu_count(),
        "load_avg": list(os.getloadavg()) if hasattr(os, "getloadavg") else None,
        "mem_total": int(vm.total), "mem_available": int(vm.available), "mem_used": int(vm.total - vm.available),
        "mem_percent": float(vm.percent),
    }
    try:
        shm = psutil.disk_usage("/dev/shm")
        s["mem_shared_bytes"] = int(shm.used)
    except Exception:
        pass
    disk = {}
    for path in {"/", session_dir or "/tmp"}:
        try:
            u = psutil.disk_usage(path)
            disk[path] = {"total": int(u.total), "used": int(u.used), "free": int(u.free), "percent": float(u.percent)}
        except Exception:
            pass
    s["disk"] = disk
    try:
        io = psutil.disk_io_counters()
        net = psutil.net_io_counters()
        s.update(disk_io_read=int(io.read_bytes), disk_io_write=int(io.write_bytes),
                 disk_io_read_count=int(io.read_count), disk_io_write_count=int(io.write_count),
                 network_sent=int(net.bytes_sent), network_received=int(net.bytes_recv))
        p = _prev_io.get("s")
        if p is not None and now > p["timestamp"]:
            dt = now - p["timestamp"]
            for k, sp in (("disk_io_read", "disk_io_read_speed"), ("disk_io_write", "disk_io_write_speed"),
                          ("network_sent", "network_send_speed"), ("network_received", "network_receive_speed")):
                s[sp] = max(0.0, (s[k] - p[k]) / dt)
        _prev_io["s"] = {k: s[k] for k in ("timestamp", "disk_io_read", "disk_io_write", "network_sent",
                                          "network_received")}
    except Exception:
        pass
    s["gpus"] = (gpus or sample_gpus)()
    return s


class NodeReporter:
    """Background sampler: ``publish(sample)`` every ``interval_s`` seconds."""

    def __init__(self, publish: Callable[[Dict[str, Any]], None], session_dir: Optional[str] = None,
                 interval_s: float = INTERVAL_S):
        self.publish = publish
        self.session_dir = session_dir
        self.interval_s = interval_s
        self._stop = threading.Event()
        self.thread: Optional[threading.Thread] = None

    def start(self) -> "NodeReporter":
        if self.interval_s > 0:
            self.thread = threading.Thread(target=self._run, name="caamd-reporter", daemon=True)
            self.thread.start()
        return self

    def _run(self):
        while not self._stop.is_set():
            try:
                self.publish(sample_node(self.session_dir))
            except Exception:
                pass
            self._stop.wait(self.interval_s)

    def stop(self):
        self._stop.set()


# ------------------------------------------------------------------ Prometheus
def prometheus_lines(nodes: List[Dict[str, Any]], session: str = "caamd") -> List[str]:
    """``ray_node_*`` gauges (reference names) for every node that has a sample."""
    from .. import __version__

    node_g = [("node_cpu_utilization", "Total CPU usage on a ray node", lambda s: s.get("cpu_percent")),
              ("node_cpu_count", "Total CPUs available on a ray node", lambda s: s.get("cpu_count")),
              ("node_mem_used", "Memory usage on a ray node", lambda s: s.get("mem_used")),
              ("node_mem_available", "Memory available on a ray node", lambda s: s.get("mem_available")),
              ("node_mem_total", "Total memory on a ray node", lambda s: s.get("mem_total")),
              ("node_mem_shared_bytes", "Total shared memory usage on a ray node", lambda s: s.get("mem_shared_bytes")),
              ("node_disk_io_read", "Total read from disk", lambda s: s.get("disk_io_read")),
              ("node_disk_io_write", "Total written to disk", lambda s: s.get("disk_io_write")),
              ("node_disk_io_read_speed", "Disk read speed", lambda s: s.get("disk_io_read_speed")),
              ("node_disk_io_write_speed", "Disk write speed", lambda s: s.get("disk_io_write_speed")),
              ("node_disk_usage", "Total disk usage (bytes) on a ray node", lambda s: (s.get("disk") or {}).get("/", {}).get("used")),
              ("node_disk_free", "Total disk free (bytes) on a ray node", lambda s: (s.get("disk") or {}).get("/", {}).get("free")),
              ("node_disk_utilization_percentage", "Total disk utilization (percentage) on a ray node",
               lambda s: (s.get("disk") or {}).get("/", {}).get("percent")),
              ("node_network_sent", "Total network sent", lambda s: s.get("network_sent")),
              ("node_network_received", "Total network received", lambda s: s.get("network_received")),
              ("node_network_send_speed", "Network send speed", lambda s: s.get("network_send_speed")),
              ("node_network_receive_speed", "Network receive speed", lambda s: s.get("network_receive_speed"))]
    gpu_g = [("node_gpus_available", "Total GPUs available on a ray node", lambda g: 1),
             ("node_gpus_utilization", "Total GPUs usage on a ray node", lambda g: g.get("utilization_gpu")),
             ("node_gram_used", "Total GPU RAM usage on a ray node", lambda g: g.get("memory_used")),
             ("node_gram_available", "Total GPU RAM available on a ray node",
              lambda g: (g["memory_total"] - g["memory_used"]) if "memory_total" in g and "memory_used" in g else None),
             ("node_gpu_power_watts", "GPU socket power", lambda g: g.get("power_w")),
             ("node_gpu_temperature_celsius", "GPU hotspot temperature", lambda g: g.get("temperature_c"))]
    rows = [(n, n.get("stats")) for n in nodes if n.get("Alive", True) and n.get("stats")]
    lines: List[str] = []

    def tags(n, extra=""):
        t = (f'ip="{n.get("NodeManagerAddress", "")}",Version="{__version__}",SessionName="{session}",'
             f'IsHeadNode="{str(bool(n.get("IsHeadNode", False))).lower()}"')
        return "{" + t + extra + "}"

    for name, desc, fn in node_g:
        vals = [(n, fn(s)) for n, s in rows]
        vals = [(n, v) for n, v in vals if v is not None]
        if not vals:
            continue
        lines += [f"# HELP ray_{name} {desc}", f"# TYPE ray_{name} gauge"]
        lines += [f"ray_{name}{tags(n)} {float(v)}" for n, v in vals]
    for name, desc, fn in gpu_g:
        vals = []
        for n, s in rows:
            for g in s.get("gpus") or []:
                v = fn(g)
                if v is not None:
                    vals.append((n, g, v))
        if not vals:
            continue
        lines += [f"# HELP ray_{name} {desc}", f"# TYPE ray_{name} gauge"]
        for n, g, v in vals:
            extra = ',GpuIndex="%s",GpuDeviceName="%s"' % (g["index"], g.get("name", ""))
            lines.append(f"ray_{name}{tags(n, extra)} {float(v)}")
    return lines
