"""``ome.io/v1beta1`` kinds as pydantic models (wire-compatible JSON/YAML field names).

Every model accepts unknown fields (``extra="allow"``) so inline Kubernetes PodSpec /
Container fields round-trip untouched, exactly as with the reference CRDs
(``pkg/apis/ome/v1beta1/*.go``).  Objects live in the store as plain dicts; controllers
parse them with :func:`parse` when they want typed access and :func:`dump` them back.
"""
from __future__ import annotations

from typing import Any, Optional

from pydantic import BaseModel as _PB
from pydantic import ConfigDict, Field
from pydantic.alias_generators import to_camel

from ome_amd.api import constants as C


class Model(_PB):
    model_config = ConfigDict(populate_by_name=True, extra="allow", alias_generator=to_camel)

    def dump(self) -> dict:
        return self.model_dump(by_alias=True, exclude_none=True, mode="json")


# ------------------------------------------------------------------ BaseModel / FT weights
class ModelFormat(Model):
    name: str
    version: Optional[str] = None
    operator: Optional[str] = None       # Equal | GreaterThan | GreaterThanOrEqual
    weight: Optional[int] = None


class ModelFrameworkSpec(ModelFormat):
    pass


class DiffusionComponentSpec(Model):
    library: Optional[str] = None
    type: Optional[str] = None


class DiffusionPipelineSpec(Model):
    class_name: Optional[str] = None
    scheduler: Optional[DiffusionComponentSpec] = None
    text_encoder: Optional[DiffusionComponentSpec] = None
    tokenizer: Optional[DiffusionComponentSpec] = None
    transformer: Optional[DiffusionComponentSpec] = None
    vae: Optional[DiffusionComponentSpec] = Field(default=None, alias="vae")
    additional_components: Optional[dict[str, DiffusionComponentSpec]] = None


class StorageSpec(Model):
    path: Optional[str] = None
    schema_path: Optional[str] = None
    parameters: Optional[dict[str, str]] = None
    storage_key: Optional[str] = Field(default=None, alias="key")
    storage_uri: Optional[str] = None
    node_selector: Optional[dict[str, str]] = None
    node_affinity: Optional[dict[str, Any]] = None
    download_policy: Optional[str] = None  # AlwaysDownload | ReuseIfExists


class BaseModelSpec(Model):
    model_format: Optional[ModelFormat] = None
    model_type: Optional[str] = None
    model_framework: Optional[ModelFrameworkSpec] = None
    model_architecture: Optional[str] = None
    quantization: Optional[str] = None     # fp8 | fbgemm_fp8 | int4
    model_parameter_size: Optional[str] = None
    model_capabilities: Optional[list[str]] = None
    api_capabilities: Optional[list[str]] = None
    model_configuration: Optional[dict[str, Any]] = None
    storage: Optional[StorageSpec] = None
    serving_mode: Optional[list[str]] = None
    max_tokens: Optional[int] = None
    diffusion_pipeline: Optional[DiffusionPipelineSpec] = None
    additional_metadata: Optional[dict[str, str]] = None
    display_name: Optional[str] = None
    version: Optional[str] = None
    disabled: Optional[bool] = None
    vendor: Optional[str] = None
    compartment_id: Optional[str] = Field(default=None, alias="compartmentID")


class ObjectReference(Model):
    name: Optional[str] = None
    namespace: Optional[str] = None


class FineTunedWeightSpec(Model):
    base_model_ref: Optional[ObjectReference] = None
    model_type: Optional[str] = None
    hyper_parameters: Optional[dict[str, Any]] = None
    configuration: Optional[dict[str, Any]] = None
    storage: Optional[StorageSpec] = None
    training_job_ref: Optional[ObjectReference] = None
    display_name: Optional[str] = None
    version: Optional[str] = None
    disabled: Optional[bool] = None
    vendor: Optional[str] = None
    compartment_id: Optional[str] = Field(default=None, alias="compartmentID")


class ModelStatusSpec(Model):
    lifecycle: Optional[str] = None
    state: str = "Creating"
    nodes_ready: Optional[list[str]] = None
    nodes_failed: Optional[list[str]] = None


class LifeCycleState:
    CREATING, IMPORTING, IN_TRANSIT, IN_TRAINING, READY, FAILED = (
        "Creating", "Importing", "In_Transit", "In_Training", "Ready", "Failed")


QUANTIZATIONS = ("fp8", "fbgemm_fp8", "int4")
MODEL_CAPABILITIES = (
    "TEXT_GENERATION", "TEXT_SUMMARIZATION", "TEXT_EMBEDDINGS", "TEXT_RERANK", "CHAT", "VISION", "EMBEDDING",
    "RERANK", "TEXT_TO_TEXT", "TEXT_TO_AUDIO", "TEXT_TO_IMAGE", "TEXT_TO_VIDEO", "IMAGE_TEXT_TO_TEXT",
    "IMAGE_TEXT_TO_AUDIO", "IMAGE_TEXT_TO_IMAGE", "IMAGE_TEXT_TO_VIDEO", "VIDEO_TEXT_TO_AUDIO", "AUDIO_TO_TEXT",
    "AUDIO_TO_AUDIO", "AUDIO_TRANSLATION")
API_CAPABILITIES = (
    "OPENAI_V1_CHAT_COMPLETIONS", "OPENAI_V1_RESPONSES", "OPENAI_V1_EMBEDDINGS", "OPENAI_V1_IMAGES_GENERATIONS",
    "OPENAI_V1_IMAGES_EDITS", "OPENAI_V1_AUDIO_SPEECH", "OPENAI_V1_AUDIO_TRANSCRIPTIONS",
    "OPENAI_V1_AUDIO_TRANSLATIONS", "OPENAI_V1_REALTIME")


# ------------------------------------------------------------------ components
class KedaAuthRef(Model):
    name: str
    kind: Optional[str] = None


class KedaConfig(Model):
    enable_keda: Optional[bool] = None
    prom_server_address: Optional[str] = None
    custom_prom_query: Optional[str] = None
    scaling_threshold: Optional[str] = None
    scaling_operator: Optional[str] = None
    authentication_ref: Optional[KedaAuthRef] = None
    auth_modes: Optional[str] = None


class ComponentExtensionSpec(Model):
    min_replicas: Optional[int] = None
    max_replicas: Optional[int] = None
    scale_target: Optional[int] = None
    scale_metric: Optional[str] = None     # cpu | memory | concurrency | rps | tps
    container_concurrency: Optional[int] = None
    timeout_seconds: Optional[int] = None
    canary_traffic_percent: Optional[int] = None
    labels: Optional[dict[str, str]] = None
    annotations: Optional[dict[str, str]] = None
    min_available: Optional[int | str] = None
    max_unavailable: Optional[int | str] = None
    deployment_strategy: Optional[dict[str, Any]] = None
    keda_config: Optional[KedaConfig] = None


class RunnerSpec(Model):
    """An inline core/v1 Container (name, image, args, env, resources, ...)."""
    name: Optional[str] = None
    image: Optional[str] = None
    command: Optional[list[str]] = None
    args: Optional[list[str]] = None
    env: Optional[list[dict[str, Any]]] = None
    resources: Optional[dict[str, Any]] = None


class PodSpecFields(Model):
    """Inline core/v1 PodSpec subset used by components (other fields pass through)."""
    containers: Optional[list[dict[str, Any]]] = None
    volumes: Optional[list[dict[str, Any]]] = None
    node_selector: Optional[dict[str, str]] = None
    affinity: Optional[dict[str, Any]] = None
    tolerations: Optional[list[dict[str, Any]]] = None
    service_account_name: Optional[str] = None
    host_ipc: Optional[bool] = Field(default=None, alias="hostIPC")
    host_network: Optional[bool] = None
    scheduler_name: Optional[str] = None
    image_pull_secrets: Optional[list[dict[str, Any]]] = None
    dns_policy: Optional[str] = None


class LeaderSpec(PodSpecFields):
    runner: Optional[RunnerSpec] = None


class WorkerSpec(PodSpecFields):
    size: Optional[int] = None
    runner: Optional[RunnerSpec] = None


class AcceleratorConstraints(Model):
    min_memory: Optional[int] = None
    max_memory: Optional[int] = None
    min_compute_performance_tflops: Optional[int] = Field(default=None, alias="minComputePerformanceTFLOPS")
    min_architecture_version: Optional[str] = None
    required_features: Optional[list[str]] = None
    excluded_classes: Optional[list[str]] = None
    architecture_families: Optional[list[str]] = None
    preferred_precisions: Optional[list[str]] = None


class AcceleratorSelector(Model):
    accelerator_class: Optional[str] = None
    constraints: Optional[AcceleratorConstraints] = None
    policy: Optional[str] = None   # BestFit | Cheapest | MostCapable | FirstAvailable


class EngineSpec(PodSpecFields, ComponentExtensionSpec):
    runner: Optional[RunnerSpec] = None
    leader: Optional[LeaderSpec] = None
    worker: Optional[WorkerSpec] = None
    accelerator_override: Optional[AcceleratorSelector] = None


class DecoderSpec(EngineSpec):
    pass


class RouterSpec(PodSpecFields, ComponentExtensionSpec):
    runner: Optional[RunnerSpec] = None
    config: Optional[dict[str, str]] = None


class ModelRef(Model):
    name: str
    kind: Optional[str] = None       # default ClusterBaseModel
    api_group: Optional[str] = None
    fine_tuned_weights: Optional[list[str]] = None


class ServingRuntimeRef(Model):
    name: str
    kind: Optional[str] = None       # ServingRuntime | ClusterServingRuntime
    api_group: Optional[str] = None


class PredictorModelSpec(Model):
    base_model: Optional[str] = None
    fine_tuned_weights: Optional[list[str]] = None
    runtime: Optional[str] = None
    protocol_version: Optional[str] = None


class PredictorSpec(PodSpecFields, ComponentExtensionSpec):
    model: Optional[PredictorModelSpec] = None
    worker_spec: Optional[WorkerSpec] = None


class InferenceServiceSpec(Model):
    predictor: Optional[PredictorSpec] = None
    engine: Optional[EngineSpec] = None
    decoder: Optional[DecoderSpec] = None
    model: Optional[ModelRef] = None
    runtime: Optional[ServingRuntimeRef] = None
    router: Optional[RouterSpec] = None
    keda_config: Optional[KedaConfig] = None
    accelerator_selector: Optional[AcceleratorSelector] = None


# ------------------------------------------------------------------ ServingRuntime
class TensorParallelismConfig(Model):
    tensor_parallel_size: Optional[int] = None
    pipeline_parallel_size: Optional[int] = None
    data_parallel_size: Optional[int] = None


class AcceleratorModelConfig(Model):
    min_memory_per_billion_params: Optional[int] = None
    tensor_parallelism_override: Optional[TensorParallelismConfig] = None
    runtime_args_override: Optional[list[str]] = None
    environment_override: Optional[dict[str, str]] = None


class SupportedModelFormat(Model):
    name: Optional[str] = None
    model_format: Optional[ModelFormat] = None
    model_type: Optional[str] = None
    version: Optional[str] = None
    model_framework: Optional[ModelFrameworkSpec] = None
    model_architecture: Optional[str] = None
    quantization: Optional[str] = None
    diffusion_pipeline: Optional[DiffusionPipelineSpec] = None
    auto_select: Optional[bool] = None
    priority: Optional[int] = None
    accelerator_config: Optional[dict[str, AcceleratorModelConfig]] = None

    def auto_select_enabled(self) -> bool:
        return bool(self.auto_select)


class ModelSizeRangeSpec(Model):
    min: Optional[str] = None
    max: Optional[str] = None


class AcceleratorRequirements(Model):
    accelerator_classes: Optional[list[str]] = None
    min_memory: Optional[int] = None
    min_compute_performance_tflops: Optional[int] = Field(default=None, alias="minComputePerformanceTFLOPS")
    min_architecture_version: Optional[str] = None
    required_features: Optional[list[str]] = None
    preferred_precisions: Optional[list[str]] = None


class WorkerPodSpec(PodSpecFields):
    size: Optional[int] = None


class ServingRuntimeSpec(PodSpecFields):
    supported_model_formats: Optional[list[SupportedModelFormat]] = None
    model_size_range: Optional[ModelSizeRangeSpec] = None
    disabled: Optional[bool] = None
    router_config: Optional[RouterSpec] = None
    engine_config: Optional[EngineSpec] = None
    decoder_config: Optional[DecoderSpec] = None
    protocol_versions: Optional[list[str]] = None
    workers: Optional[WorkerPodSpec] = None
    accelerator_requirements: Optional[AcceleratorRequirements] = None
    labels: Optional[dict[str, str]] = None
    annotations: Optional[dict[str, str]] = None

    def is_disabled(self) -> bool:
        return bool(self.disabled)

    def supports_protocol(self, proto: str | None) -> bool:
        return not proto or not self.protocol_versions or proto in self.protocol_versions

    def supports_accelerator_class(self, ac: str) -> bool:
        req = self.accelerator_requirements
        return req is None or not req.accelerator_classes or ac in req.accelerator_classes

    def priority_of(self, fmt_name: str) -> int | None:
        for f in self.supported_model_formats or []:
            if f.name == fmt_name:
                return f.priority
        return None


# ------------------------------------------------------------------ AcceleratorClass
class AcceleratorDiscovery(Model):
    node_selector: Optional[dict[str, str]] = None
    affinity: Optional[dict[str, Any]] = None
    pci_vendor_id: Optional[str] = Field(default=None, alias="pciVendorID")
    device_ids: Optional[list[str]] = Field(default=None, alias="deviceIDs")


class AcceleratorLatency(Model):
    average_millis: Optional[int] = None
    maximum_millis: Optional[int] = None


class AcceleratorPerformance(Model):
    fp32_tflops: Optional[int] = Field(default=None, alias="fp32Tflops")
    fp16_tflops: Optional[int] = Field(default=None, alias="fp16Tflops")
    int8_tops: Optional[int] = Field(default=None, alias="int8Tops")
    int4_tops: Optional[int] = Field(default=None, alias="int4Tops")
    latency: Optional[AcceleratorLatency] = None


class AcceleratorCapabilities(Model):
    memory_gb: Optional[str | int | float] = Field(default=None, alias="memoryGB")
    compute_capability: Optional[str] = None
    level_zero_version: Optional[str] = None
    clock_speed_mhz: Optional[int] = Field(default=None, alias="clockSpeedMHz")
    memory_bandwidth_gbps: Optional[str | int | float] = Field(default=None, alias="memoryBandwidthGBps")
    features: Optional[list[str]] = None
    performance: Optional[AcceleratorPerformance] = None


class AcceleratorResource(Model):
    name: str
    quantity: Optional[str | int] = None
    divisible: Optional[bool] = None


class AcceleratorIntegration(Model):
    kueue_resource_flavor: Optional[str] = None
    volcano_gpu_type: Optional[str] = Field(default=None, alias="volcanoGPUType")


class AcceleratorCost(Model):
    per_hour: Optional[str | int | float] = None
    per_million_tokens: Optional[str | int | float] = None
    spot_per_hour: Optional[str | int | float] = None
    tier: Optional[str] = None


class AcceleratorClassSpec(Model):
    vendor: Optional[str] = None
    family: Optional[str] = None
    model: Optional[str] = None
    discovery: AcceleratorDiscovery = Field(default_factory=AcceleratorDiscovery)
    capabilities: AcceleratorCapabilities = Field(default_factory=AcceleratorCapabilities)
    resources: Optional[list[AcceleratorResource]] = None
    integration: Optional[AcceleratorIntegration] = None
    cost: Optional[AcceleratorCost] = None


# ------------------------------------------------------------------ BenchmarkJob
class InferenceServiceReference(Model):
    name: str
    namespace: str


class Endpoint(Model):
    url: str = Field(alias="url")
    api_format: str
    model_name: Optional[str] = None


class EndpointSpec(Model):
    inference_service: Optional[InferenceServiceReference] = None
    endpoint: Optional[Endpoint] = None


class ServiceMetadata(Model):
    engine: str
    version: str
    gpu_type: str
    gpu_count: int


class PodOverride(Model):
    image: Optional[str] = None
    env: Optional[list[dict[str, Any]]] = None
    env_from: Optional[list[dict[str, Any]]] = None
    volume_mounts: Optional[list[dict[str, Any]]] = None
    resources: Optional[dict[str, Any]] = None
    tolerations: Optional[list[dict[str, Any]]] = None
    node_selector: Optional[dict[str, str]] = None
    affinity: Optional[dict[str, Any]] = None
    volumes: Optional[list[dict[str, Any]]] = None


class HuggingFaceSecretReference(Model):
    name: str


class BenchmarkJobSpec(Model):
    hugging_face_secret_reference: Optional[HuggingFaceSecretReference] = None
    endpoint: EndpointSpec
    service_metadata: Optional[ServiceMetadata] = None
    task: str
    traffic_scenarios: Optional[list[str]] = None
    num_concurrency: Optional[list[int]] = None
    max_time_per_iteration: Optional[int] = None
    max_requests_per_iteration: Optional[int] = None
    additional_request_params: Optional[dict[str, str]] = None
    dataset: Optional[StorageSpec] = None
    output_location: Optional[StorageSpec] = None
    result_folder_name: Optional[str] = None
    pod_override: Optional[PodOverride] = None


# ------------------------------------------------------------------ kinds
KINDS = {
    # kind: (plural, namespaced, spec model)
    "BaseModel": ("basemodels", True, BaseModelSpec),
    "ClusterBaseModel": ("clusterbasemodels", False, BaseModelSpec),
    "FineTunedWeight": ("finetunedweights", False, FineTunedWeightSpec),
    "ServingRuntime": ("servingruntimes", True, ServingRuntimeSpec),
    "ClusterServingRuntime": ("clusterservingruntimes", False, ServingRuntimeSpec),
    "InferenceService": ("inferenceservices", True, InferenceServiceSpec),
    "AcceleratorClass": ("acceleratorclasses", False, AcceleratorClassSpec),
    "BenchmarkJob": ("benchmarkjobs", True, BenchmarkJobSpec),
}
SHORT_NAMES = {"isvc": "InferenceService", "bm": "BaseModel", "cbm": "ClusterBaseModel", "sr": "ServingRuntime",
               "csr": "ClusterServingRuntime", "ac": "AcceleratorClass", "bj": "BenchmarkJob",
               "ftw": "FineTunedWeight"}


def spec_of(obj: dict):
    """Typed spec of a stored ome.io object."""
    return KINDS[obj["kind"]][2].model_validate(obj.get("spec") or {})


def dump(model: Model) -> dict:
    return model.dump()


def new_object(kind: str, name: str, namespace: str | None = None, spec: dict | Model | None = None,
               labels: dict | None = None, annotations: dict | None = None) -> dict:
    meta: dict[str, Any] = {"name": name}
    if KINDS.get(kind, (None, True))[1] and namespace:
        meta["namespace"] = namespace
    if labels:
        meta["labels"] = dict(labels)
    if annotations:
        meta["annotations"] = dict(annotations)
    sp = spec.dump() if isinstance(spec, Model) else (spec or {})
    return {"apiVersion": C.API_VERSION, "kind": kind, "metadata": meta, "spec": sp}
