"""Controller configuration from the ``ome/inferenceservice-config`` and ``ome/benchmarkjob-config``
ConfigMaps (keys ``ingress``, ``deploy``, ``metricsAggregator``, ``modelInit``,
``multinodeProber``, ``kedaConfig``, ``benchmarkjob``), re-read on every reconcile like the
reference (``pkg/controller/v1beta1/controllerconfig/configmap.go``).  Missing keys fall back
to the defaults shipped in ``config/configmap/inferenceservice.yaml``.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, fields

from ome_amd.api import constants as C
from ome_amd.store.store import Store


@dataclass
class IngressConfig:
    ingressGateway: str = "knative-serving/knative-ingress-gateway"
    ingressService: str = "istio-ingressgateway.istio-system.svc.cluster.local"
    localGateway: str = "knative-serving/knative-local-gateway"
    localGatewayService: str = "knative-local-gateway.istio-system.svc.cluster.local"
    omeIngressGateway: str = ""
    ingressDomain: str = "svc.cluster.local"
    ingressClassName: str = "istio"
    additionalIngressDomains: list | None = None
    domainTemplate: str = "{{ .Name }}.{{ .Namespace }}.{{ .IngressDomain }}"
    urlScheme: str = "http"
    disableIstioVirtualHost: bool = False
    pathTemplate: str = ""
    disableIngressCreation: bool = True
    enableGatewayAPI: bool = False


@dataclass
class DeployConfig:
    defaultDeploymentMode: str = C.DeploymentMode.RAW


@dataclass
class MultiNodeProberConfig:
    image: str = "ome-amd/multinode-prober:latest"
    memoryRequest: str = "100Mi"
    memoryLimit: str = "100Mi"
    cpuRequest: str = "100m"
    cpuLimit: str = "100m"
    startupFailureThreshold: int = 150
    startupPeriodSeconds: int = 30
    startupTimeoutSeconds: int = 60
    startupInitialDelaySeconds: int = 200
    unavailableThresholdSeconds: int = 1800


@dataclass
class MetricsAggregatorConfig:
    enableMetricAggregation: str = "false"
    enablePrometheusScraping: str = "false"


@dataclass
class ModelInitConfig:
    image: str = "ome-amd/ome-agent:latest"
    memoryRequest: str = "16Gi"
    memoryLimit: str = "16Gi"
    cpuRequest: str = "4"
    cpuLimit: str = "4"
    compartmentId: str = ""
    authType: str = "InstancePrincipal"
    vaultId: str = ""
    region: str = ""


@dataclass
class KedaDefaults:
    enableKeda: bool = True
    promServerAddress: str = "http://prometheus-operated.monitoring.svc.cluster.local:9090"
    customPromQuery: str = ""
    scalingThreshold: str = "10"
    scalingOperator: str = "GreaterThanOrEqual"


@dataclass
class BenchmarkJobConfig:
    podConfig: dict = field(default_factory=lambda: {
        "image": "ome-amd/loadgen:latest", "cpuRequest": "2", "memoryRequest": "2Gi", "cpuLimit": "2",
        "memoryLimit": "2Gi"})


def _load(cls, raw: str | None):
    obj = cls()
    if not raw:
        return obj
    try:
        data = json.loads(raw)
    except json.JSONDecodeError as e:
        raise ValueError(f"invalid JSON in config key for {cls.__name__}: {e}") from e
    names = {f.name for f in fields(cls)}
    for k, v in (data or {}).items():
        if k in names:
            setattr(obj, k, v)
    return obj


@dataclass
class ControllerConfig:
    ingress: IngressConfig
    deploy: DeployConfig
    prober: MultiNodeProberConfig
    metrics: MetricsAggregatorConfig
    model_init: ModelInitConfig
    keda: KedaDefaults
    benchmark: BenchmarkJobConfig

    @classmethod
    def from_store(cls, store: Store, namespace: str = C.OME_NAMESPACE) -> "ControllerConfig":
        cm = store.try_get("v1", "ConfigMap", C.INFERENCESERVICE_CONFIGMAP, namespace) or {}
        data = cm.get("data") or {}
        bcm = store.try_get("v1", "ConfigMap", C.BENCHMARKJOB_CONFIGMAP, namespace) or {}
        return cls(ingress=_load(IngressConfig, data.get("ingress")), deploy=_load(DeployConfig, data.get("deploy")),
                   prober=_load(MultiNodeProberConfig, data.get("multinodeProber")),
                   metrics=_load(MetricsAggregatorConfig, data.get("metricsAggregator")),
                   model_init=_load(ModelInitConfig, data.get("modelInit")),
                   keda=_load(KedaDefaults, data.get("kedaConfig")),
                   benchmark=_load(BenchmarkJobConfig, (bcm.get("data") or {}).get("benchmarkjob")))


def resolve_ingress(cfg: IngressConfig, annotations: dict | None) -> IngressConfig:
    """Per-ISVC ``ome.io/ingress-*`` annotation overrides (``utils/annotations.go:93``)."""
    import dataclasses

    a = annotations or {}
    out = dataclasses.replace(cfg)
    if C.INGRESS_DOMAIN_TEMPLATE in a:
        out.domainTemplate = a[C.INGRESS_DOMAIN_TEMPLATE]
    if C.INGRESS_DOMAIN in a:
        out.ingressDomain = a[C.INGRESS_DOMAIN]
    if C.INGRESS_ADDITIONAL_DOMAINS in a:
        out.additionalIngressDomains = [d.strip() for d in a[C.INGRESS_ADDITIONAL_DOMAINS].split(",") if d.strip()]
    if C.INGRESS_URL_SCHEME in a:
        out.urlScheme = a[C.INGRESS_URL_SCHEME]
    if C.INGRESS_PATH_TEMPLATE in a:
        out.pathTemplate = a[C.INGRESS_PATH_TEMPLATE]
    if C.INGRESS_DISABLE_ISTIO_VIRTUALHOST in a:
        out.disableIstioVirtualHost = a[C.INGRESS_DISABLE_ISTIO_VIRTUALHOST].lower() == "true"
    if C.INGRESS_DISABLE_CREATION in a:
        out.disableIngressCreation = a[C.INGRESS_DISABLE_CREATION].lower() == "true"
    return out


def render_template(tmpl: str, values: dict) -> str:
    """Tiny Go-template subset: ``{{ .Field }}`` and ``{{ .Labels.key }}`` / ``{{ .Annotations.key }}``."""
    import re

    def sub(m):
        path = m.group(1).split(".")
        cur = values
        for p in path:
            if isinstance(cur, dict) and p in cur:
                cur = cur[p]
            else:
                return ""
        return str(cur)

    return re.sub(r"\{\{\s*\.([A-Za-z0-9_.\-/]+)\s*\}\}", sub, tmpl)
