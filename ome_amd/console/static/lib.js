// ome-amd web console — DOM-free helpers shared by the views (and unit-tested under node by
// tests/test_console_js_cpu.py): escaping, a YAML emitter for the manifest previews, CSV/JSON
// export, sorting, the storage-URI builder/parser (grammar of ome_amd/storage/uri.py, the
// reference's pkg/utils/storage/storage.go) and the manifest builders behind the structured forms
// (reference web-console/frontend/src/lib/validation/{model,runtime}-schema.ts and
// components/forms/*: the same fields, emitted as ClusterBaseModel / ClusterServingRuntime /
// InferenceService / BenchmarkJob objects).
"use strict";
(function (root) {
  const nz = (a, b) => (a === null || a === undefined ? b : a);   // (kept node-12 compatible: no ?? / ?.)
  const esc = (s) => String(nz(s, "")).replace(/[&<>"']/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;" }[c]));

  // ------------------------------------------------------------------ YAML (block style, for previews)
  const PLAIN = /^[A-Za-z_/][A-Za-z0-9_./@:+-]*$/;
  const RESERVED = new Set(["true", "false", "null", "yes", "no", "on", "off", "~", ""]);
  function scalar(v) {
    if (v === null || v === undefined) return "null";
    if (typeof v === "boolean" || typeof v === "number") return String(v);
    const s = String(v);
    if (PLAIN.test(s) && !RESERVED.has(s.toLowerCase()) && !/^[0-9.+-]/.test(s) && !s.includes(": ")) return s;
    return JSON.stringify(s);   // a JSON string is a valid YAML double-quoted scalar
  }
  function isEmpty(v) { return v && typeof v === "object" && Object.keys(v).length === 0; }
  function toYaml(v, ind = 0) {
    const pad = " ".repeat(ind);
    if (Array.isArray(v)) {
      if (!v.length) return "[]";
      return v.map((x) => {
        if (x && typeof x === "object" && !isEmpty(x)) {
          const body = toYaml(x, ind + 2);
          return `${pad}- ${body.slice(ind + 2)}`;
        }
        return `${pad}- ${x && typeof x === "object" ? (Array.isArray(x) ? "[]" : "{}") : scalar(x)}`;
      }).join("\n");
    }
    if (v && typeof v === "object") {
      const keys = Object.keys(v).filter((k) => v[k] !== undefined);
      if (!keys.length) return "{}";
      return keys.map((k) => {
        const x = v[k];
        if (x && typeof x === "object" && !isEmpty(x)) {
          return Array.isArray(x) ? `${pad}${scalar(k)}:\n${toYaml(x, ind)}` : `${pad}${scalar(k)}:\n${toYaml(x, ind + 2)}`;
        }
        return `${pad}${scalar(k)}: ${x && typeof x === "object" ? (Array.isArray(x) ? "[]" : "{}") : scalar(x)}`;
      }).join("\n");
    }
    return pad + scalar(v);
  }

  // ------------------------------------------------------------------ export / sort
  function csvCell(v) {
    const s = v === null || v === undefined ? "" : typeof v === "object" ? JSON.stringify(v) : String(v);
    return /[",\n]/.test(s) ? `"${s.replace(/"/g, '""')}"` : s;
  }
  function toCsv(cols, rows) {   // cols: [[header, (row) => value], ...]
    return [cols.map((c) => csvCell(c[0])).join(","), ...rows.map((r) => cols.map((c) => csvCell(c[1](r))).join(","))].join("\n") + "\n";
  }
  function get(o, path) { return path.split(".").reduce((a, k) => (a == null ? undefined : a[k]), o); }
  function cmp(a, b) {
    const na = typeof a === "number" ? a : parseSize(a), nb = typeof b === "number" ? b : parseSize(b);
    if (na !== null && nb !== null && !Number.isNaN(na) && !Number.isNaN(nb)) return na - nb;
    return String(nz(a, "")).localeCompare(String(nz(b, "")), undefined, { numeric: true });
  }
  function sortRows(rows, key, dir = 1) { return [...rows].sort((x, y) => dir * cmp(key(x), key(y))); }
  // "7B", "1.5B", "480M", "2T" -> parameters; plain numbers stay numbers; anything else -> null
  function parseSize(s) {
    if (s === null || s === undefined || s === "") return null;
    const m = /^\s*([0-9]*\.?[0-9]+)\s*([KMBT]?)\s*$/i.exec(String(s));
    if (!m) return null;
    return parseFloat(m[1]) * ({ "": 1, K: 1e3, M: 1e6, B: 1e9, T: 1e12 }[m[2].toUpperCase()]);
  }
  function ago(ts, now = Date.now()) {
    const t = Date.parse(ts || "");
    if (Number.isNaN(t)) return "";
    const s = Math.max(0, Math.round((now - t) / 1000));
    return s < 60 ? `${s}s` : s < 3600 ? `${Math.floor(s / 60)}m` : s < 86400 ? `${Math.floor(s / 3600)}h` : `${Math.floor(s / 86400)}d`;
  }
  function fmtBytes(n) {
    n = Number(n || 0);
    const u = ["B", "KiB", "MiB", "GiB", "TiB"];
    let i = 0;
    while (n >= 1024 && i < u.length - 1) { n /= 1024; i++; }
    return `${n.toFixed(i ? 1 : 0)} ${u[i]}`;
  }

  // ------------------------------------------------------------------ storage URIs
  const SCHEMES = {
    hf: { label: "Hugging Face", fields: [["repo", "meta-llama/Llama-3.1-8B-Instruct"], ["revision", "main (optional)"]] },
    oci: { label: "OCI Object Storage", fields: [["namespace", "my-namespace"], ["bucket", "my-bucket"], ["prefix", "models/my-model"]] },
    s3: { label: "Amazon S3", fields: [["bucket", "my-bucket"], ["region", "us-west-2 (optional)"], ["prefix", "models/my-model"]] },
    az: { label: "Azure Blob", fields: [["account", "mystorageaccount"], ["container", "models"], ["path", "my-model/v1"]] },
    gs: { label: "Google Cloud Storage", fields: [["bucket", "my-bucket"], ["object", "models/my-model"]] },
    pvc: { label: "PersistentVolumeClaim", fields: [["namespace", "(optional)"], ["claim", "model-storage"], ["subpath", "models/my-model"]] },
    github: { label: "GitHub release", fields: [["repo", "owner/repo"], ["tag", "latest (optional)"]] },
    vendor: { label: "Vendor", fields: [["vendor", "my-vendor"], ["type", "models"], ["path", "my-model"]] },
    local: { label: "Local path", fields: [["path", "/raid/models/meta-llama/llama-3.1-8b-instruct"]] },
    random: { label: "Random-init weights (synthetic)", fields: [["preset", "llama-3-8b"], ["layers", "(optional)"]] },
  };
  function buildUri(scheme, f) {
    const t = (k) => String(nz(f[k], "")).trim();
    switch (scheme) {
      case "hf": return `hf://${t("repo")}${t("revision") ? "@" + t("revision") : ""}`;
      case "oci": return `oci://n/${t("namespace")}/b/${t("bucket")}/o/${t("prefix")}`;
      case "s3": return `s3://${t("bucket")}${t("region") ? "@" + t("region") : ""}/${t("prefix")}`;
      case "az": return `az://${t("account")}/${t("container")}/${t("path")}`;
      case "gs": return `gs://${t("bucket")}/${t("object")}`;
      case "pvc": return `pvc://${t("namespace") ? t("namespace") + ":" : ""}${t("claim")}/${t("subpath")}`;
      case "github": return `github://${t("repo")}${t("tag") ? "@" + t("tag") : ""}`;
      case "vendor": return `vendor://${t("vendor")}/${t("type")}/${t("path")}`;
      case "local": return `local://${t("path").replace(/^local:\/\//, "")}`;
      case "random": return `random://${t("preset")}${t("layers") ? "?layers=" + t("layers") : ""}`;
    }
    throw new Error(`unknown storage scheme ${scheme}`);
  }
  function parseUri(uri) {
    const m = /^([a-z0-9]+):\/\/(.*)$/.exec(String(uri || "").trim());
    if (!m || !SCHEMES[m[1]]) return null;
    const [, scheme, rest] = m;
    let r;
    switch (scheme) {
      case "hf": { const [repo, revision] = rest.split("@"); r = { repo, revision: revision || "" }; break; }
      case "oci": {
        const o = /^n\/([^/]+)\/b\/([^/]+)\/o\/(.*)$/.exec(rest);
        if (!o) return null;
        r = { namespace: o[1], bucket: o[2], prefix: o[3] }; break;
      }
      case "s3": {
        const i = rest.indexOf("/"), head = i < 0 ? rest : rest.slice(0, i), [bucket, region] = head.split("@");
        r = { bucket, region: region || "", prefix: i < 0 ? "" : rest.slice(i + 1) }; break;
      }
      case "az": {
        const p = rest.split("/");
        r = { account: p[0].replace(/\.blob\.core\.windows\.net$/, ""), container: p[1] || "", path: p.slice(2).join("/") }; break;
      }
      case "gs": { const i = rest.indexOf("/"); r = { bucket: i < 0 ? rest : rest.slice(0, i), object: i < 0 ? "" : rest.slice(i + 1) }; break; }
      case "pvc": {
        const i = rest.indexOf("/"), head = i < 0 ? rest : rest.slice(0, i), c = head.indexOf(":");
        r = { namespace: c < 0 ? "" : head.slice(0, c), claim: c < 0 ? head : head.slice(c + 1), subpath: i < 0 ? "" : rest.slice(i + 1) }; break;
      }
      case "github": { const [repo, tag] = rest.split("@"); r = { repo, tag: tag || "" }; break; }
      case "vendor": { const p = rest.split("/"); r = { vendor: p[0], type: p[1] || "", path: p.slice(2).join("/") }; break; }
      case "local": r = { path: rest }; break;
      case "random": { const [preset, q] = rest.split("?"); r = { preset, layers: (/layers=(\d+)/.exec(q || "") || [])[1] || "" }; break; }
    }
    return { scheme, fields: r };
  }

  // ------------------------------------------------------------------ manifest builders
  const API_VERSION = "ome.io/v1beta1";
  const NAME_RE = /^[a-z]([-a-z0-9]*[a-z0-9])?$/;
  const prune = (o) => {   // drop "", undefined, empty objects/arrays (forms leave many fields blank)
    if (Array.isArray(o)) { const a = o.map(prune).filter((x) => x !== undefined); return a.length ? a : undefined; }
    if (o && typeof o === "object") {
      const r = {};
      for (const [k, v] of Object.entries(o)) { const p = prune(v); if (p !== undefined) r[k] = p; }
      return Object.keys(r).length ? r : undefined;
    }
    return o === "" || o === undefined || o === null || (typeof o === "number" && Number.isNaN(o)) ? undefined : o;
  };
  function kvObject(pairs) {   // [[k, v], ...] -> {k: v} (blank keys dropped)
    const r = {};
    for (const [k, v] of pairs || []) if (String(k || "").trim()) r[String(k).trim()] = String(nz(v, ""));
    return r;
  }
  function validateName(n, what = "name") {
    if (!n) return `${what} is required`;
    if (n.length > 63) return `${what} must be at most 63 characters`;
    if (!NAME_RE.test(n)) return `${what} must be lower-case alphanumeric or '-', start with a letter and end alphanumeric`;
    return null;
  }
  function buildModel(f) {
    const storage = {
      storageUri: f.storageUri, path: f.path, key: f.storageKey,
      nodeSelector: kvObject(f.nodeSelector), parameters: kvObject(f.parameters),
    };
    const spec = {
      vendor: f.vendor, displayName: f.displayName, version: f.version, disabled: f.disabled || undefined,
      modelFormat: { name: f.formatName, version: f.formatVersion },
      modelFramework: { name: f.frameworkName, version: f.frameworkVersion },
      modelArchitecture: f.architecture, modelParameterSize: f.parameterSize, quantization: f.quantization,
      modelCapabilities: f.capabilities, maxTokens: f.maxTokens ? Number(f.maxTokens) : undefined, storage,
    };
    const obj = { apiVersion: API_VERSION, kind: f.namespace ? "BaseModel" : "ClusterBaseModel",
                  metadata: { name: f.name, namespace: f.namespace || undefined, labels: kvObject(f.labels) }, spec };
    const out = prune(obj);
    out.spec = out.spec || {};
    if (f.huggingFaceToken) out.huggingFaceToken = f.huggingFaceToken;
    return out;
  }
  function modelErrors(f) {
    const e = [];
    const n = validateName(f.name); if (n) e.push(n);
    if (!f.storageUri) e.push("storage URI is required");
    else if (!parseUri(f.storageUri) && !String(f.storageUri).startsWith("/")) e.push(`unsupported storage URI ${f.storageUri}`);
    if (f.parameterSize && parseSize(f.parameterSize) === null) e.push("parameter size must look like 7B, 1.5B or 480M");
    if (f.maxTokens && !(Number(f.maxTokens) > 0)) e.push("max tokens must be a positive number");
    return e;
  }
  function container(c) {
    if (!c) return undefined;
    const split = (s) => (Array.isArray(s) ? s : String(s || "").split(/\s+/)).filter(Boolean);
    return prune({
      name: c.name || "ome-container", image: c.image, command: split(c.command), args: split(c.args),
      env: (c.env || []).filter(([k]) => k).map(([name, value]) => ({ name, value: String(nz(value, "")) })),
      resources: { requests: prune({ cpu: c.cpu, memory: c.memory }), limits: prune({ cpu: c.cpuLimit, memory: c.memoryLimit, "amd.com/gpu": c.gpus ? String(c.gpus) : undefined }) },
      ports: c.port ? [{ containerPort: Number(c.port), name: "http1", protocol: "TCP" }] : undefined,
      volumeMounts: (c.mounts || []).filter((m) => m.name && m.mountPath).map((m) => ({ name: m.name, mountPath: m.mountPath, readOnly: m.readOnly || undefined })),
    });
  }
  function buildRuntime(f) {
    const formats = (f.formats || []).map((x) => prune({
      name: x.name || x.formatName, modelFormat: { name: x.formatName, version: x.formatVersion },
      modelFramework: { name: x.frameworkName, version: x.frameworkVersion }, modelArchitecture: x.architecture,
      quantization: x.quantization, autoSelect: !!x.autoSelect, priority: x.priority === "" || x.priority === undefined ? undefined : Number(x.priority),
    }));
    const engine = {};
    if (f.multiNode) {
      engine.leader = { runner: container(f.engine) };
      engine.worker = { size: Number(f.workers || 1), runner: container(f.worker || f.engine) };
    } else {
      engine.runner = container(f.engine);
    }
    const spec = {
      disabled: f.disabled || undefined, supportedModelFormats: formats, protocolVersions: f.protocols,
      modelSizeRange: prune({ min: f.sizeMin, max: f.sizeMax }), engineConfig: engine,
      decoderConfig: f.decoder ? { runner: container(f.decoder) } : undefined,
      routerConfig: f.router ? { runner: container(f.router) } : undefined,
      acceleratorRequirements: f.accelerators && f.accelerators.length ? { acceleratorClasses: f.accelerators } : undefined,
      volumes: (f.volumes || []).filter((v) => v.name).map((v) => v.claim ? { name: v.name, persistentVolumeClaim: { claimName: v.claim } }
        : v.hostPath ? { name: v.name, hostPath: { path: v.hostPath } } : { name: v.name, emptyDir: v.medium ? { medium: v.medium } : {} }),
    };
    return prune({ apiVersion: API_VERSION, kind: f.namespace ? "ServingRuntime" : "ClusterServingRuntime",
                   metadata: { name: f.name, namespace: f.namespace || undefined, labels: kvObject(f.labels) }, spec });
  }
  function runtimeErrors(f) {
    const e = [];
    const n = validateName(f.name); if (n) e.push(n);
    if (!(f.formats || []).length) e.push("at least one supported model format is required");
    (f.formats || []).forEach((x, i) => {
      if (!x.formatName) e.push(`format #${i + 1}: format name is required`);
      if (x.autoSelect && (x.priority === "" || x.priority === undefined)) e.push(`format #${i + 1}: priority is required when autoSelect is on`);
      if (x.priority !== "" && x.priority !== undefined && !(Number(x.priority) >= 0)) e.push(`format #${i + 1}: priority must be >= 0`);
    });
    if (f.sizeMin && parseSize(f.sizeMin) === null) e.push("model size min must look like 1B");
    if (f.sizeMax && parseSize(f.sizeMax) === null) e.push("model size max must look like 70B");
    if (f.sizeMin && f.sizeMax && parseSize(f.sizeMin) > parseSize(f.sizeMax)) e.push("model size min is larger than max");
    if (!f.engine || !f.engine.image) e.push("engine image is required");
    if (f.multiNode && !(Number(f.workers) > 0)) e.push("multi-node runtimes need workers.size > 0");
    return e;
  }
  function buildService(f) {
    const ann = {};
    if (f.autoscaler) ann["ome.io/autoscalerClass"] = f.autoscaler;
    if (f.autoscaler === "hpa" && f.metric) ann["ome.io/metrics"] = f.metric;
    if (f.target) ann["ome.io/targetUtilizationPercentage"] = String(f.target);
    if (f.deploymentMode) ann["ome.io/deploymentMode"] = f.deploymentMode;
    const comp = (min, max) => prune({ minReplicas: min === "" ? undefined : Number(min), maxReplicas: max === "" ? undefined : Number(max) });
    const spec = {
      model: { name: f.model, kind: f.modelNamespaced ? "BaseModel" : undefined },
      runtime: f.runtime ? { name: f.runtime } : undefined,
      engine: { ...(comp(nz(f.min, 1), nz(f.max, 1)) || {}), runner: f.gpus || (f.env && f.env.length) ? container({ gpus: f.gpus, env: f.env }) : undefined },
      decoder: f.pd ? comp(nz(f.dmin, 1), nz(f.dmax, 1)) || {} : undefined,
      router: f.pd || f.router ? comp(1, 1) : undefined,
      kedaConfig: f.autoscaler === "keda" ? prune({ enableKeda: true, promServerAddress: f.promServer, customPromQuery: f.promQuery,
                                                   scalingThreshold: f.threshold, scalingOperator: f.operator }) : undefined,
    };
    const obj = prune({ apiVersion: API_VERSION, kind: "InferenceService",
                        metadata: { name: f.name, namespace: f.namespace || "default", annotations: ann }, spec });
    if (f.pd && obj.spec && !obj.spec.decoder) obj.spec.decoder = {};
    if (obj.spec && !obj.spec.engine) obj.spec.engine = {};
    return obj;
  }
  function serviceErrors(f) {
    const e = [];
    const n = validateName(f.name, "service name"); if (n) e.push(n);
    if (!f.model) e.push("model is required");
    if (f.min !== "" && f.max !== "" && Number(f.min) > Number(f.max)) e.push("min replicas exceed max replicas");
    if (f.target && !(Number(f.target) >= 1 && Number(f.target) <= 100)) e.push("target utilisation must be in [1-100]");
    if (f.autoscaler === "hpa" && f.metric && !["cpu", "memory"].includes(f.metric)) e.push(`[${f.metric}] is not a supported metric`);
    if (f.autoscaler === "keda" && f.operator && !["GreaterThanOrEqual", "LessThanOrEqual"].includes(f.operator)) e.push("invalid KEDA scaling operator");
    return e;
  }
  function buildBenchmark(f) {
    const endpoint = f.url ? { endpoint: { url: f.url, apiFormat: f.apiFormat || "openai", modelName: f.modelName } }
      : { inferenceService: { name: f.service, namespace: f.serviceNamespace || f.namespace || "default" } };
    // scenarios contain commas (N(480,240)/(300,150)): split them on whitespace / ';' only
    const list = (s, re = /[\s,;]+/) => (Array.isArray(s) ? s : String(s || "").split(re)).filter(Boolean);
    return prune({
      apiVersion: API_VERSION, kind: "BenchmarkJob", metadata: { name: f.name, namespace: f.namespace || "default" },
      spec: {
        endpoint, task: f.task || "text-to-text", trafficScenarios: list(f.scenarios, /[\s;]+/), numConcurrency: list(f.concurrency).map(Number),
        maxTimePerIteration: f.maxTime ? Number(f.maxTime) : undefined, maxRequestsPerIteration: f.maxRequests ? Number(f.maxRequests) : undefined,
        outputLocation: f.output ? { storageUri: f.output } : undefined,
      },
    });
  }
  // GitHub blob URL or catalog-relative path -> path under the console's catalog roots
  function catalogPath(s) {
    s = String(s || "").trim();
    const m = /^https?:\/\/(?:github\.com\/[^/]+\/[^/]+\/(?:blob|raw)\/[^/]+|raw\.githubusercontent\.com\/[^/]+\/[^/]+\/[^/]+)\/(.*)$/.exec(s);
    return m ? m[1] : s;
  }

  const OME = { esc, toYaml, toCsv, get, cmp, sortRows, parseSize, ago, fmtBytes, SCHEMES, buildUri, parseUri, prune, kvObject,
                validateName, buildModel, modelErrors, buildRuntime, runtimeErrors, container, buildService, serviceErrors,
                buildBenchmark, catalogPath, API_VERSION };
  if (typeof module !== "undefined" && module.exports) module.exports = OME;
  root.OME = OME;
})(typeof globalThis !== "undefined" ? globalThis : this);
