"""``python -m cluster_anywhere_amd.autoscaler.monitor --address HEAD:PORT --config cfg.yaml``:
standalone autoscaler process with the local node provider (reference:
autoscaler/_private/monitor.py)."""
from __future__ import annotations

import argparse
import time


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--interval", type=float, default=5.0)
    a = ap.parse_args(argv)
    import signal

    def _term(*_):
        raise KeyboardInterrupt  # `down` sends SIGTERM: terminate our node agents first

    signal.signal(signal.SIGTERM, _term)
    from ..core import api
    from .autoscaler import Monitor, StandardAutoscaler
    from .node_provider import LocalNodeProvider

    api.init(address=a.address)
    prov = LocalNodeProvider(a.address)
    mon = Monitor(StandardAutoscaler(a.config, prov), a.interval).start()
    try:
        while True:
            time.sleep(a.interval)
            print(mon.autoscaler.summary(), flush=True)
    except KeyboardInterrupt:
        pass
    finally:
        mon.stop()
        prov.shutdown()


if __name__ == "__main__":
    main()
