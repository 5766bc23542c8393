"""Status types and whole-object envelopes of the ``ome.io/v1beta1`` kinds.

The spec models live in :mod:`ome_amd.api.v1beta1`; this module adds what the reference's Go
types carry around them (``pkg/apis/ome/v1beta1/*_status.go``, ``inference_service_status.go``,
``benchmark_types.go``, ``accelerator_class_types.go``): the status blocks the controllers
write, the legacy predictor ``ModelSpec`` / extension specs, and for every kind the typed
``<Kind>`` (apiVersion / kind / metadata / spec / status) and ``<Kind>List`` envelopes.  These
are what :mod:`ome_amd.api.openapi` publishes as ``v1beta1.*`` definitions and what the Python
SDK (:mod:`ome_amd.sdk`) returns.
"""
from __future__ import annotations

from typing import Any, Optional

from pydantic import Field, create_model

from ome_amd.api import constants as C
from ome_amd.api import v1beta1 as V
from ome_amd.api.v1beta1 import Model


# ------------------------------------------------------------------ shared
class Condition(Model):
    """knative ``apis.Condition`` as the status blocks carry it."""
    type: str
    status: str = "Unknown"                # True | False | Unknown
    severity: Optional[str] = None
    last_transition_time: Optional[str] = None
    reason: Optional[str] = None
    message: Optional[str] = None


class Addressable(Model):
    url: Optional[str] = None


class TrafficTarget(Model):
    revision_name: Optional[str] = None
    latest_revision: Optional[bool] = None
    percent: Optional[int] = None
    tag: Optional[str] = None
    url: Optional[str] = None


# ------------------------------------------------------------------ InferenceService status
class AcceleratorSelection(Model):
    accelerator_class: str
    node_selector: Optional[dict[str, str]] = None
    resource_requests: Optional[dict[str, Any]] = None
    reason: Optional[str] = None


class ComponentStatusSpec(Model):
    latest_ready_revision: Optional[str] = None
    latest_created_revision: Optional[str] = None
    previous_rolledout_revision: Optional[str] = None
    latest_rolledout_revision: Optional[str] = None
    traffic: Optional[list[TrafficTarget]] = None
    url: Optional[str] = None
    rest_url: Optional[str] = Field(default=None, alias="restURL")
    address: Optional[Addressable] = None
    selected_accelerator: Optional[AcceleratorSelection] = None


class FailureInfo(Model):
    location: Optional[str] = None
    reason: Optional[str] = None           # ModelLoadFailed | RuntimeUnhealthy | NoSupportingRuntime | ...
    message: Optional[str] = None
    model_revision_name: Optional[str] = None
    time: Optional[str] = None
    exit_code: Optional[int] = None


class ModelCopies(Model):
    failed_copies: int = 0
    total_copies: Optional[int] = None


class ModelRevisionStates(Model):
    active_model_state: str = ""           # Pending | Standby | Loading | Loaded | FailedToLoad
    target_model_state: Optional[str] = None


class ModelStatus(Model):
    transition_status: str = ""            # UpToDate | InProgress | BlockedByFailedLoad | InvalidSpec
    model_revision_states: Optional[ModelRevisionStates] = None
    last_failure_info: Optional[FailureInfo] = None
    model_copies: Optional[ModelCopies] = None


class InferenceServiceStatus(Model):
    observed_generation: Optional[int] = None
    conditions: Optional[list[Condition]] = None
    annotations: Optional[dict[str, str]] = None
    url: Optional[str] = None
    address: Optional[Addressable] = None
    components: Optional[dict[str, ComponentStatusSpec]] = None
    model_status: Optional[ModelStatus] = None


# ------------------------------------------------------------------ other statuses
class BenchmarkJobStatus(Model):
    state: str = "Pending"                 # Pending | Running | Completed | Failed
    start_time: Optional[str] = None
    completion_time: Optional[str] = None
    last_reconcile_time: Optional[str] = None
    failure_message: Optional[str] = None
    details: Optional[str] = None


class AcceleratorClassStatus(Model):
    nodes: Optional[list[str]] = None
    total_accelerators: Optional[int] = None
    available_accelerators: Optional[int] = None
    available_nodes: Optional[int] = None
    last_updated: Optional[str] = None
    conditions: Optional[list[Condition]] = None


class ServingRuntimeStatus(Model):
    """Empty in the reference too (runtimes are configuration, not reconciled objects)."""


class ScalerAuthenticationRef(V.KedaAuthRef):
    """KEDA ``TriggerAuthentication`` reference (the reference's name for ``KedaAuthRef``)."""


class SupportedRuntime(Model):
    """A (name, spec) pair the runtime selector returns."""
    name: str = Field(alias="Name")
    spec: V.ServingRuntimeSpec = Field(alias="Spec")


# ------------------------------------------------------------------ pod / container specs
_CONTAINER = dict(
    name=(Optional[str], None), image=(Optional[str], None), command=(Optional[list[str]], None),
    args=(Optional[list[str]], None), working_dir=(Optional[str], None), ports=(Optional[list[dict[str, Any]]], None),
    env=(Optional[list[dict[str, Any]]], None), env_from=(Optional[list[dict[str, Any]]], None),
    resources=(Optional[dict[str, Any]], None), resize_policy=(Optional[list[dict[str, Any]]], None),
    restart_policy=(Optional[str], None), volume_mounts=(Optional[list[dict[str, Any]]], None),
    volume_devices=(Optional[list[dict[str, Any]]], None), liveness_probe=(Optional[dict[str, Any]], None),
    readiness_probe=(Optional[dict[str, Any]], None), startup_probe=(Optional[dict[str, Any]], None),
    lifecycle=(Optional[dict[str, Any]], None), termination_message_path=(Optional[str], None),
    termination_message_policy=(Optional[str], None), image_pull_policy=(Optional[str], None),
    security_context=(Optional[dict[str, Any]], None), stdin=(Optional[bool], None),
    stdin_once=(Optional[bool], None), tty=(Optional[bool], None),
)
PredictorExtensionSpec = create_model(
    "PredictorExtensionSpec", __base__=Model, __doc__="Container fields + storage / protocol of a legacy predictor.",
    storage_uri=(Optional[str], None), runtime_version=(Optional[str], None), protocol_version=(Optional[str], None),
    **_CONTAINER)
ModelSpec = create_model(
    "ModelSpec", __base__=PredictorExtensionSpec, __doc__="Legacy predictor model: base model, weights, runtime.",
    base_model=(Optional[str], None), fine_tuned_weights=(Optional[list[str]], None), runtime=(Optional[str], None))
ModelExtensionSpec = create_model(
    "ModelExtensionSpec", __base__=Model, __doc__="Display / ownership fields shared by model kinds.",
    display_name=(Optional[str], None), version=(Optional[str], None), disabled=(Optional[bool], None),
    vendor=(Optional[str], None), compartment_id=(Optional[str], Field(default=None, alias="compartmentID")))


class PodSpec(V.PodSpecFields):
    """core/v1 PodSpec: the commonly set fields typed, the rest passed through (``extra=allow``)."""
    init_containers: Optional[list[dict[str, Any]]] = None
    restart_policy: Optional[str] = None
    termination_grace_period_seconds: Optional[int] = None
    service_account: Optional[str] = None
    hostname: Optional[str] = None
    subdomain: Optional[str] = None
    priority_class_name: Optional[str] = None
    runtime_class_name: Optional[str] = None
    topology_spread_constraints: Optional[list[dict[str, Any]]] = None
    security_context: Optional[dict[str, Any]] = None
    host_pid: Optional[bool] = Field(default=None, alias="hostPID")


class ServingRuntimePodSpec(V.PodSpecFields):
    labels: Optional[dict[str, str]] = None
    annotations: Optional[dict[str, str]] = None


# ------------------------------------------------------------------ object envelopes
STATUS_OF = {
    "BaseModel": V.ModelStatusSpec, "ClusterBaseModel": V.ModelStatusSpec, "FineTunedWeight": V.ModelStatusSpec,
    "ServingRuntime": ServingRuntimeStatus, "ClusterServingRuntime": ServingRuntimeStatus,
    "InferenceService": InferenceServiceStatus, "AcceleratorClass": AcceleratorClassStatus,
    "BenchmarkJob": BenchmarkJobStatus,
}


class ObjectMeta(Model):
    name: Optional[str] = None
    namespace: Optional[str] = None
    labels: Optional[dict[str, str]] = None
    annotations: Optional[dict[str, str]] = None
    uid: Optional[str] = None
    resource_version: Optional[str] = None
    generation: Optional[int] = None
    creation_timestamp: Optional[str] = None
    deletion_timestamp: Optional[str] = None
    finalizers: Optional[list[str]] = None
    owner_references: Optional[list[dict[str, Any]]] = None


class ListMeta(Model):
    resource_version: Optional[str] = None
    continue_: Optional[str] = Field(default=None, alias="continue")


def _envelope(kind: str):
    spec = V.KINDS[kind][2]
    obj = create_model(kind, __base__=Model, __doc__=f"``{C.API_VERSION}`` {kind}.",
                       api_version=(str, Field(default=C.API_VERSION, alias="apiVersion")),
                       kind=(str, kind), metadata=(ObjectMeta, Field(default_factory=ObjectMeta)),
                       spec=(spec, Field(default_factory=spec) if not _required(spec) else ...),
                       status=(Optional[STATUS_OF[kind]], None))
    lst = create_model(f"{kind}List", __base__=Model, __doc__=f"List of {kind}.",
                       api_version=(str, Field(default=C.API_VERSION, alias="apiVersion")),
                       kind=(str, f"{kind}List"), metadata=(Optional[ListMeta], None), items=(list[obj], []))
    return obj, lst


def _required(model) -> bool:
    return any(f.is_required() for f in model.model_fields.values())


OBJECTS: dict[str, type] = {}
LISTS: dict[str, type] = {}
for _k in V.KINDS:
    OBJECTS[_k], LISTS[_k] = _envelope(_k)
    globals()[_k], globals()[f"{_k}List"] = OBJECTS[_k], LISTS[_k]


def parse(obj: dict):
    """Typed envelope of a stored object (the spec validated; unknown fields kept)."""
    return OBJECTS[obj["kind"]].model_validate(obj)


def parse_list(kind: str, body: dict):
    return LISTS[kind].model_validate(body)
