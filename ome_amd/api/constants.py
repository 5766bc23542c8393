"""Names, labels, annotations and naming helpers of the ``ome.io/v1beta1`` API.

Kept wire-compatible with the reference so manifests written for it keep working
(``pkg/constants/constants.go``); deliberate deviations are marked.
"""
from __future__ import annotations

import hashlib
import os

GROUP = "ome.io"
VERSION = "v1beta1"
API_VERSION = f"{GROUP}/{VERSION}"
OME_NAMESPACE = os.environ.get("POD_NAMESPACE", "ome")

# ConfigMaps
INFERENCESERVICE_CONFIGMAP = "inferenceservice-config"
BENCHMARKJOB_CONFIGMAP = "benchmarkjob-config"

# Finalizers
ISVC_FINALIZER = "inferenceservice.finalizers"
BASEMODEL_FINALIZER = "basemodels.ome.io/finalizer"
CLUSTERBASEMODEL_FINALIZER = "clusterbasemodels.ome.io/finalizer"
ACCELERATORCLASS_FINALIZER = "acceleratorclasses.ome.io/finalizer"
BENCHMARKJOB_FINALIZER = "benchmarkjob.ome.io/finalizer"

# Annotations (ISVC)
DEPLOYMENT_MODE = f"{GROUP}/deploymentMode"
AUTOSCALER_CLASS = f"{GROUP}/autoscalerClass"
AUTOSCALER_METRICS = f"{GROUP}/metrics"
TARGET_UTILIZATION = f"{GROUP}/targetUtilizationPercentage"
DEPRECATION_WARNING = f"{GROUP}/deprecation-warning"
MODEL_INIT_INJECTION = f"{GROUP}/inject-model-init"
FT_ADAPTER_INJECTION = f"{GROUP}/inject-fine-tuned-adapter"
SERVING_SIDECAR_INJECTION = f"{GROUP}/inject-serving-sidecar"
ENABLE_METRIC_AGGREGATION = f"{GROUP}/enable-metric-aggregation"
ENABLE_PROMETHEUS_SCRAPING = f"{GROUP}/enable-prometheus-scraping"
BASE_MODEL_NAME_ANN = f"{GROUP}/base-model-name"
BASE_MODEL_VENDOR_ANN = f"{GROUP}/base-model-vendor"
BASE_MODEL_FORMAT_ANN = f"{GROUP}/base-model-format"
BASE_MODEL_FORMAT_VERSION_ANN = f"{GROUP}/base-model-format-version"
SERVING_RUNTIME_ANN = f"{GROUP}/serving-runtime"
ENTRYPOINT_COMPONENT = f"{GROUP}/entrypoint-component"
SERVICE_TYPE = f"{GROUP}/service-type"
LOAD_BALANCER_IP = f"{GROUP}/load-balancer-ip"
DEDICATED_AI_CLUSTER = f"{GROUP}/dedicated-ai-cluster"
VOLCANO_QUEUE_ANN = f"{GROUP}/volcano-queue"
INGRESS_DOMAIN_TEMPLATE = f"{GROUP}/ingress-domain-template"
INGRESS_DOMAIN = f"{GROUP}/ingress-domain"
INGRESS_ADDITIONAL_DOMAINS = f"{GROUP}/ingress-additional-domains"
INGRESS_URL_SCHEME = f"{GROUP}/ingress-url-scheme"
INGRESS_PATH_TEMPLATE = f"{GROUP}/ingress-path-template"
INGRESS_DISABLE_ISTIO_VIRTUALHOST = f"{GROUP}/ingress-disable-istio-virtualhost"
INGRESS_DISABLE_CREATION = f"{GROUP}/ingress-disable-creation"
BASE_MODEL_DECRYPTION_KEY = f"{GROUP}/base-model-decryption-key-name"
BASE_MODEL_DECRYPTION_SECRET = f"{GROUP}/base-model-decryption-secret-name"
DISABLE_MODEL_DECRYPTION = f"{GROUP}/disable-model-decryption"
PROMETHEUS_SCRAPE = "prometheus.io/scrape"
PROMETHEUS_PORT = "prometheus.io/port"
PROMETHEUS_PATH = "prometheus.io/path"
CONTAINER_PROMETHEUS_PORT = "prometheus.ome.io/port"
CONTAINER_PROMETHEUS_PATH = "prometheus.ome.io/path"
DEFAULT_PROMETHEUS_PATH = "/metrics"
# RDMA / interconnect injection.  The reference's profile targets 16x mlx5 RoCE HCAs
# (oci-roce); on an 8xMI355X node the fabric is xGMI, so our default profile is amd-xgmi.
RDMA_AUTO_INJECT = "rdma.ome.io/auto-inject"
RDMA_PROFILE = "rdma.ome.io/profile"
RDMA_CONTAINER_NAME = "rdma.ome.io/container-name"
KEDA_THRESHOLD = "autoscaling.keda.sh/threshold"
KEDA_OPERATOR = "autoscaling.keda.sh/operator"
KEDA_SERVER_ADDRESS = "autoscaling.keda.sh/prometheus.serverAddress"
KEDA_QUERY = "autoscaling.keda.sh/prometheus.query"
RAY_UNAVAILABLE_SINCE = "raycluster/unavailable-since"
MODEL_CATEGORY = "models.ome.io/category"
SKIP_CONFIG_PARSING = "ome.oracle.com/skip-config-parsing"
RESERVE_MODEL_ARTIFACT = "models.ome/reserve-model-artifact"
TARGET_INSTANCE_SHAPES = "models.ome.io/target-instance-shapes"

# Labels
ISVC_LABEL = f"{GROUP}/inferenceservice"
COMPONENT_LABEL = "component"
ENDPOINT_LABEL = "endpoint"
SERVING_RUNTIME_LABEL = "serving-runtime"
BASE_MODEL_NAME_LABEL = "base-model-name"
BASE_MODEL_SIZE_LABEL = "base-model-size"
BASE_MODEL_TYPE_LABEL = "base-model-type"
BASE_MODEL_VENDOR_LABEL = "base-model-vendor"
FT_SERVING_LABEL = "fine-tuned-serving"
MODEL_STATUS_CM_LABEL = "models.ome/basemodel-status"
MODEL_LABEL_DOMAIN = "models.ome.io"
CLUSTER_BASE_MODEL_LABEL_TYPE = "clusterbasemodel"
BASE_MODEL_LABEL_TYPE = "basemodel"
RAW_APP_LABEL = "app"
LWS_WORKER_INDEX_LABEL = "leaderworkerset.sigs.k8s.io/worker-index"
LWS_NAME_LABEL = "leaderworkerset.sigs.k8s.io/name"
RAY_NODE_TYPE_LABEL = "ray.io/node-type"
ISTIO_SIDECAR_INJECT = "sidecar.istio.io/inject"
KUEUE_QUEUE_LABEL = "kueue.x-k8s.io/queue-name"
KUEUE_PRIORITY_LABEL = "kueue.x-k8s.io/priority-class"
VOLCANO_QUEUE_LABEL = "volcano.sh/queue-name"
NODE_INSTANCE_TYPE_LABEL = "node.kubernetes.io/instance-type"

# Components / protocols / ports
PREDICTOR, ROUTER, ENGINE, DECODER = "predictor", "router", "engine", "decoder"
OPENAI_PROTOCOL = "openAI"
OPEN_INFERENCE_V1 = "openInference-v1"
OPEN_INFERENCE_V2 = "openInference-v2"
DEFAULT_HTTP_PORT = 8080
MAIN_CONTAINER = "ome-container"
MULTINODE_PROBER_CONTAINER = "multinode-prober"
MODEL_INIT_CONTAINER = "model-init"
FT_ADAPTER_CONTAINER = "fine-tuned-adapter"
SERVING_SIDECAR_CONTAINER = "serving-sidecar"

# Env contract to engine pods
MODEL_PATH_ENV = "MODEL_PATH"
SERVED_MODEL_NAME_ENV = "SERVED_MODEL_NAME"
PARALLELISM_SIZE_ENV = "PARALLELISM_SIZE"
LWS_LEADER_ADDRESS_ENV = "LWS_LEADER_ADDRESS"
LWS_GROUP_SIZE_ENV = "LWS_GROUP_SIZE"
LWS_WORKER_INDEX_ENV = "LWS_WORKER_INDEX"

# GPU resources.  The reference hardcodes nvidia.com/gpu (constants.go:258); here the
# resource name is configurable and defaults to AMD's device-plugin resource.
AMD_GPU_RESOURCE = "amd.com/gpu"
NVIDIA_GPU_RESOURCE = "nvidia.com/gpu"
GPU_RESOURCE = os.environ.get("OME_GPU_RESOURCE", AMD_GPU_RESOURCE)
GPU_RESOURCE_NAMES = (AMD_GPU_RESOURCE, NVIDIA_GPU_RESOURCE)

DEFAULT_MODEL_LOCAL_MOUNT_PATH = "/mnt/models"


class DeploymentMode:
    SERVERLESS = "Serverless"
    RAW = "RawDeployment"
    MULTINODE_RAY_VLLM = "MultiNodeRayVLLM"
    PD = "PDDisaggregated"
    MULTINODE = "MultiNode"
    VIRTUAL = "VirtualDeployment"
    ALL = (SERVERLESS, RAW, MULTINODE_RAY_VLLM, PD, MULTINODE, VIRTUAL)

    @classmethod
    def is_valid(cls, m: str) -> bool:
        return m in cls.ALL


AUTOSCALER_HPA, AUTOSCALER_KEDA, AUTOSCALER_EXTERNAL = "hpa", "keda", "external"
AUTOSCALER_CLASSES = (AUTOSCALER_HPA, AUTOSCALER_KEDA, AUTOSCALER_EXTERNAL)
AUTOSCALER_METRICS_ALLOWED = ("cpu", "memory")
DEFAULT_CPU_UTILIZATION = 80

# Kubernetes naming limits
MAX_LABEL_NAME_LENGTH = 49  # 63 - len("models.ome.io") - 1
MAX_CONFIGMAP_KEY_LENGTH = 253
HASH_PREFIX_LENGTH = 8


# ---------------------------------------------------------------------- naming helpers
def _hash8(s: str) -> str:
    return hashlib.sha256(s.encode()).hexdigest()[:HASH_PREFIX_LENGTH]


def truncate_with_hash(original: str, max_len: int, dns_safe: bool = False) -> str:
    """``{sha256[:8]}-{suffix}`` when too long (suffix keeps the most specific part)."""
    if len(original) <= max_len:
        return original
    h = _hash8(original)
    if dns_safe and h[0].isdigit():
        h = "a" + h[1:]
    suffix_len = max_len - HASH_PREFIX_LENGTH - 1
    if suffix_len <= 0:
        return h[:max_len]
    return f"{h}-{original[len(original) - suffix_len:]}"


def truncate_name(name: str, max_len: int) -> str:
    return truncate_with_hash(name, max_len, dns_safe=True)


def _split_ns_model(namespace: str, model: str, available: int) -> tuple[str, str]:
    if len(namespace) + len(model) <= available:
        return namespace, model
    min_len = 8
    if available < 2 * min_len:
        ns_max = available // 2
        m_max = available - ns_max
    elif len(namespace) <= min_len:
        ns_max = len(namespace)
        m_max = available - ns_max
    else:
        ns_max = min_len
        m_max = available - ns_max
    return truncate_with_hash(namespace, ns_max), truncate_with_hash(model, m_max)


def cluster_base_model_label(model: str) -> str:
    """``models.ome.io/clusterbasemodel.<name>`` (node readiness label key)."""
    mx = MAX_LABEL_NAME_LENGTH - len(CLUSTER_BASE_MODEL_LABEL_TYPE) - 1
    return f"{MODEL_LABEL_DOMAIN}/{CLUSTER_BASE_MODEL_LABEL_TYPE}.{truncate_with_hash(model, mx)}"


def base_model_label(namespace: str, model: str) -> str:
    """``models.ome.io/<ns>.basemodel.<name>``."""
    avail = MAX_LABEL_NAME_LENGTH - (len(BASE_MODEL_LABEL_TYPE) + 1) - 1
    ns, m = _split_ns_model(namespace, model, avail)
    return f"{MODEL_LABEL_DOMAIN}/{ns}.{BASE_MODEL_LABEL_TYPE}.{m}"


def model_label(namespace: str | None, model: str, cluster: bool) -> str:
    return cluster_base_model_label(model) if cluster else base_model_label(namespace or "", model)


def model_configmap_key(namespace: str | None, model: str, cluster: bool) -> str:
    if cluster:
        mx = MAX_CONFIGMAP_KEY_LENGTH - len(CLUSTER_BASE_MODEL_LABEL_TYPE) - 1
        return f"{CLUSTER_BASE_MODEL_LABEL_TYPE}.{truncate_with_hash(model, mx)}"
    avail = MAX_CONFIGMAP_KEY_LENGTH - (len(BASE_MODEL_LABEL_TYPE) + 1) - 1
    ns, m = _split_ns_model(namespace or "", model, avail)
    return f"{ns}.{BASE_MODEL_LABEL_TYPE}.{m}"


def parse_model_configmap_key(key: str) -> tuple[str, str, bool] | None:
    """-> (namespace, model, is_cluster) or None."""
    p = CLUSTER_BASE_MODEL_LABEL_TYPE + "."
    if key.startswith(p):
        return "", key[len(p):], True
    sep = f".{BASE_MODEL_LABEL_TYPE}."
    if sep in key:
        ns, m = key.split(sep, 1)
        return ns, m, False
    return None


def modelconfig_name(isvc: str) -> str:
    return f"modelconfig-{isvc[-20:]}"


def lws_name(isvc: str) -> str:
    return f"lws-{isvc[-50:]}"


def engine_name(isvc: str) -> str:
    return f"{isvc}-engine"


def decoder_name(isvc: str) -> str:
    return f"{isvc}-decoder"


def router_name(isvc: str) -> str:
    return f"{isvc}-router"


def component_name(isvc: str, component: str) -> str:
    return isvc if component == PREDICTOR else f"{isvc}-{component}"


def isvc_host(name: str, namespace: str, domain: str) -> str:
    return f"{name}.{namespace}.{domain}"


def ray_head_service_name(name: str, index: int) -> str:
    return truncate_name(f"{name}-{index}", 50)
