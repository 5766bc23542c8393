"""Web console: REST backend + single-page dashboard.

``python -m ome_amd.console --manager http://127.0.0.1:9443`` runs it standalone against a
manager; ``python -m ome_amd.manager`` also serves it in-process under ``/console``.
"""
from ome_amd.console.api import create_app, create_router, mount  # noqa: F401
