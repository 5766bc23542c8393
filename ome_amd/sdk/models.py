"""SDK model classes under the generated SDK's names (``V1beta1<Type>``, one per ``v1beta1.<Type>``
definition of :mod:`ome_amd.api.openapi`).  They are the pydantic models themselves, so
``V1beta1InferenceService.model_validate(d)`` / ``.dump()`` round-trip the wire format."""
from __future__ import annotations

from pydantic import BaseModel as _PB

from ome_amd.api import objects as _O
from ome_amd.api import v1beta1 as _V

__all__: list[str] = []


def _export(mod) -> None:
    for name, val in vars(mod).items():
        if isinstance(val, type) and issubclass(val, _PB) and val is not _V.Model and not name.startswith("_"):
            alias = f"V1beta1{name}"
            if alias not in globals():
                globals()[alias] = val
                __all__.append(alias)


_export(_V)
_export(_O)
