"""Standalone web console: ``python -m ome_amd.console [--manager URL | --catalog PATH ...]``.

With ``--manager`` the console is its own process over the manager's REST API (the reference
deploys the console as a separate Deployment next to the kube-apiserver); without it an
in-process store is created and the ``--catalog`` YAMLs are applied (demo / air-gapped review).
"""
from __future__ import annotations

import argparse
import logging


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="ome-amd web console")
    ap.add_argument("--manager", default=None, help="manager REST base URL (e.g. http://127.0.0.1:9443)")
    ap.add_argument("--catalog", action="append", default=[], help="YAML file/dir to load into an in-process store")
    ap.add_argument("--catalog-root", action="append", default=None, help="directories fetch-yaml may read")
    ap.add_argument("--models-root", default=None, help="model-agent download root (offline HF lookups)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=3000)
    ap.add_argument("--cors-origin", action="append", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ome_amd.console.api import create_app

    if a.manager:
        from ome_amd.console.remote import RemoteStore

        store = RemoteStore(a.manager)
    else:
        from ome_amd.manager import Cluster

        cl = Cluster(with_agent=False, with_executor=False)
        for c in a.catalog:
            cl.load_catalog(c)
        store = cl.store
    import uvicorn

    uvicorn.run(create_app(store, a.catalog_root, a.models_root, a.cors_origin), host=a.host, port=a.port,
                log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
