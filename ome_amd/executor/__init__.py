"""Local node executor: turns the workload objects the controllers create (Deployment,
LeaderWorkerSet, Job, Knative Service, RayCluster, HPA/ScaledObject, Service, Ingress) into
supervised processes on one MI355X node.  See :mod:`.kubelet` and :mod:`.workloads`."""
from __future__ import annotations

import glob
import os
import threading

from ome_amd.controllers.runtime import Manager
from ome_amd.executor.autoscaler import MetricsAutoscaler
from ome_amd.executor.kubelet import Kubelet, NodeInfo
from ome_amd.executor.workloads import controllers as workload_controllers
from ome_amd.store.store import Store


def detect_gpus() -> int:
    """Count gfx GPUs from the KFD topology (no HIP init — safe before fork/exec)."""
    env = os.environ.get("OME_NODE_GPUS")
    if env:
        return int(env)
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                txt = f.read()
        except OSError:
            continue
        for line in txt.splitlines():
            if line.startswith("simd_count") and int(line.split()[1]) > 0:
                n += 1
    return n or 8


class NodeExecutor:
    def __init__(self, store: Store, manager: Manager | None = None, node_name: str = "mi355x-node-0",
                 gpus: int | None = None, state_dir: str = "/tmp/ome-executor", simulate: bool = False,
                 node_labels: dict | None = None, sync_period: float = 0.5, probe_scale: float = 1.0,
                 autoscale_period: float = 15.0):
        self.store = store
        self.manager = manager or Manager(store)
        self.kubelet = Kubelet(store, NodeInfo(node_name, gpus if gpus is not None else detect_gpus(),
                                               node_labels or {}), state_dir, simulate=simulate,
                               probe_scale=probe_scale)
        for c in workload_controllers(store):
            self.manager.add(c)
        self.autoscaler = MetricsAutoscaler(store, self.kubelet, autoscale_period)
        self.sync_period = sync_period
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def step(self, rounds: int = 3) -> None:
        """Synchronous drive for tests: controllers to idle, one kubelet sync, repeat."""
        for _ in range(rounds):
            self.manager.run_until_idle(fast_forward=2.0)
            self.kubelet.sync()
        self.manager.run_until_idle(fast_forward=2.0)

    def _loop(self) -> None:
        while not self._stop.wait(self.sync_period):
            try:
                self.kubelet.sync()
            except Exception:  # noqa: BLE001
                import logging

                logging.getLogger("ome_amd.executor").exception("kubelet sync failed")

    def start(self) -> None:
        self._thread = threading.Thread(target=self._loop, name="kubelet", daemon=True)
        self._thread.start()
        self.manager.add_runnable(self.autoscaler.run)

    def shutdown(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        self.kubelet.shutdown()


__all__ = ["NodeExecutor", "Kubelet", "NodeInfo", "detect_gpus"]
