// ome-amd web console — hash-routed single-page app over the console REST API (api/v1).
"use strict";
const API = "api/v1";
const $ = (s, el = document) => el.querySelector(s);
const $$ = (s, el = document) => [...el.querySelectorAll(s)];
const esc = (s) => String(s ?? "").replace(/[&<>"]/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;" }[c]));
const enc = encodeURIComponent;

async function j(path, opt) {
  const r = await fetch(`${API}${path}`, opt);
  const body = await r.json().catch(() => ({}));
  if (!r.ok) throw new Error(typeof body.detail === "object" ? (body.detail.details || body.detail.error || JSON.stringify(body.detail))
                                                              : (body.detail || JSON.stringify(body)));
  return body;
}
const send = (method, path, obj, type = "application/json") =>
  j(path, { method, headers: { "Content-Type": type }, body: typeof obj === "string" ? obj : JSON.stringify(obj) });
const post = (p, o, t) => send("POST", p, o, t);
const put = (p, o, t) => send("PUT", p, o, t);
const del = (p) => j(p, { method: "DELETE" });

// ---------------------------------------------------------------- helpers
function ready(o) {
  const st = o.status || {};
  if (st.state) return st.state;
  const c = (st.conditions || []).find((c) => c.type === "Ready");
  return c ? (c.status === "True" ? "Ready" : c.status === "False" ? "NotReady" : "Unknown") : "-";
}
function badge(s) {
  const cls = ["Ready", "True", "Completed", "Succeeded"].includes(s) ? "ok" : ["Failed", "False", "NotReady"].includes(s) ? "bad" : "warn";
  return `<span class="${cls}">${esc(s)}</span>`;
}
function table(cols, rows, href) {
  if (!rows.length) return `<p class="muted">none</p>`;
  return `<table><tr>${cols.map((c) => `<th>${c[0]}</th>`).join("")}</tr>` + rows.map((r) =>
    `<tr class="${href ? "click" : ""}" ${href ? `data-href="${esc(href(r))}"` : ""}>${cols.map((c) => `<td>${c[1](r)}</td>`).join("")}</tr>`).join("") + "</table>";
}
function wire() { $$("#page tr[data-href]").forEach((tr) => tr.onclick = () => { location.hash = tr.dataset.href; }); }
function kv(pairs) { return `<div class="kv">${pairs.map(([k, v]) => `<div>${esc(k)}</div><div>${v}</div>`).join("")}</div>`; }
function page(html) { $("#page").innerHTML = html; wire(); }
function showErr(e, where = "#page") { $(where).insertAdjacentHTML("afterbegin", `<div class="err">${esc(e.message || e)}</div>`); }
function filterBox(id) { return `<input id="${id}" placeholder="filter…" size="24">`; }
function applyFilter(id) {
  const inp = $(`#${id}`);
  if (!inp) return;
  inp.oninput = () => $$("#page tr.click").forEach((tr) => { tr.style.display = tr.textContent.toLowerCase().includes(inp.value.toLowerCase()) ? "" : "none"; });
}
function jsonEditor(obj) {
  const o = JSON.parse(JSON.stringify(obj));
  if (o.metadata) { for (const k of ["uid", "creationTimestamp", "generation", "managedFields"]) delete o.metadata[k]; }
  return `<textarea id="ed">${esc(JSON.stringify(o, null, 2))}</textarea>`;
}

// ---------------------------------------------------------------- dashboard
async function Dashboard() {
  const [sum, svcs, models] = await Promise.all([j("/summary"), j("/services"), j("/models")]);
  const card = (label, c, href) => `<a class="card" href="#${href}"><b>${c.ready ?? c}/${c.total ?? c}</b><span>${label}</span></a>`;
  page(`<h2>Dashboard</h2><div class="cards">
      ${card("base models ready", sum.models, "models")}${card("services ready", sum.services, "services")}
      <a class="card" href="#runtimes"><b>${sum.runtimes.total}</b><span>serving runtimes</span></a>
      <a class="card" href="#accelerators"><b>${sum.accelerators.total}</b><span>accelerator classes</span></a>
      <a class="card" href="#benchmarks"><b>${sum.benchmarks.total}</b><span>benchmark jobs</span></a>
      <div class="card"><b>${sum.nodes}</b><span>nodes</span></div></div>
    <h3>Inference services</h3>${table([["namespace/name", (s) => esc(`${s.metadata.namespace}/${s.metadata.name}`)],
      ["model", (s) => esc(s.spec?.model?.name)], ["state", (s) => badge(ready(s))], ["url", (s) => esc(s.status?.url || "")]],
      svcs.items, (s) => `services/${s.metadata.namespace}/${s.metadata.name}`)}
    <h3>Models not ready</h3>${table([["name", (m) => esc(m.metadata.name)], ["state", (m) => badge(ready(m))],
      ["storage", (m) => esc(m.spec?.storage?.storageUri)]], models.items.filter((m) => ready(m) !== "Ready"), (m) => `models/${m.metadata.name}`)}`);
}

// ---------------------------------------------------------------- models
async function ModelList() {
  const { items } = await j("/models");
  page(`<h2>Cluster base models (${items.length})</h2><div class="row">${filterBox("mf")}
      <a class="btn" href="#models/new">new model</a><a class="btn sec" href="#models/import">import from Hugging Face</a></div>` +
    table([["name", (m) => esc(m.metadata.name)], ["vendor", (m) => esc(m.spec?.vendor)], ["arch", (m) => esc(m.spec?.modelArchitecture)],
      ["size", (m) => esc(m.spec?.modelParameterSize)], ["format", (m) => esc(m.spec?.modelFormat?.name)],
      ["capabilities", (m) => (m.spec?.modelCapabilities || []).map((c) => `<span class="pill">${esc(c)}</span>`).join("")],
      ["state", (m) => badge(ready(m))], ["nodes", (m) => esc((m.status?.nodesReady || []).length)]], items, (m) => `models/${m.metadata.name}`));
  applyFilter("mf");
}
async function ModelDetail(name) {
  const [m, prog, ev] = await Promise.all([j(`/models/${enc(name)}`), j(`/models/${enc(name)}/progress`), j(`/models/${enc(name)}/events`)]);
  const rec = await j(`/runtimes/recommend?model=${enc(name)}`).catch((e) => ({ error: e.message }));
  const compat = await j(`/runtimes/compatible?model=${enc(name)}`).catch(() => ({ runtimes: [] }));
  const bars = (prog.progress || []).map((p) => `<div>${esc(p.node)} · ${esc(p.phase)} ${Number(p.percentage || 0).toFixed(1)}%
      <div class="bar"><i style="width:${Number(p.percentage || 0)}%"></i></div></div>`).join("") || `<p class="muted">no download in progress</p>`;
  page(`<h2>${esc(name)} ${badge(ready(m))}</h2><div class="row"><a class="btn sec" href="#models/${enc(name)}/edit">edit</a>
      <a class="btn sec" href="#services/deploy?model=${enc(name)}">deploy</a><button class="btn" id="del">delete</button></div>` +
    kv([["storage", esc(m.spec?.storage?.storageUri)], ["path", esc(m.spec?.storage?.path)], ["architecture", esc(m.spec?.modelArchitecture)],
      ["parameters", esc(m.spec?.modelParameterSize)], ["format", esc(`${m.spec?.modelFormat?.name || ""} ${m.spec?.modelFormat?.version || ""}`)],
      ["quantization", esc(m.spec?.quantization || "")], ["nodes ready", esc((m.status?.nodesReady || []).join(", "))],
      ["nodes failed", esc((m.status?.nodesFailed || []).join(", "))],
      ["recommended runtime", rec.runtime ? `<a href="#runtimes/${enc(rec.runtime)}">${esc(rec.runtime)}</a> (score ${esc(rec.score)})` : esc(rec.error || "-")]]) +
    `<h3>Download progress</h3>${bars}<h3>Compatible runtimes</h3>` +
    table([["runtime", (r) => esc(r.runtime)], ["score", (r) => esc(r.score)], ["why", (r) => esc((r.reasons || []).join("; "))]],
      compat.runtimes || [], (r) => `runtimes/${r.runtime}`) +
    `<h3>Events</h3>${(ev.events || []).map((e) => `<div class="muted">${esc(e.reason)}: ${esc(e.message)}</div>`).join("") || "<p class='muted'>none</p>"}
     <h3>Object</h3><pre>${esc(JSON.stringify(m, null, 2))}</pre>`);
  $("#del").onclick = async () => { if (confirm(`delete ${name}?`)) { try { await del(`/models/${enc(name)}`); location.hash = "models"; } catch (e) { showErr(e); } } };
}
function ModelNew() {
  page(`<h2>New cluster base model</h2>
    <label>name</label><input id="n" size="40" placeholder="llama-3-8b-instruct">
    <label>storage URI</label><input id="u" size="60" placeholder="hf://meta-llama/Meta-Llama-3-8B-Instruct · oci://n/ns/b/bucket/o/path · s3://bucket/prefix · random://llama-3-8b">
    <label>local path on nodes (optional)</label><input id="p" size="60" placeholder="/raid/models/...">
    <label>format</label><select id="f"><option>safetensors</option><option>pytorch</option><option>gguf</option></select>
    <label>vendor</label><input id="v" size="20">
    <label>node selector (key=value, optional)</label><input id="ns" size="40">
    <div class="row"><button class="btn" id="val">validate</button><button class="btn" id="go">create</button></div><pre id="out"></pre>`);
  const obj = () => {
    const st = { storageUri: $("#u").value };
    if ($("#p").value) st.path = $("#p").value;
    if ($("#ns").value.includes("=")) { const [k, v] = $("#ns").value.split("="); st.nodeSelector = { [k.trim()]: v.trim() }; }
    return { metadata: { name: $("#n").value }, spec: { vendor: $("#v").value || undefined, modelFormat: { name: $("#f").value }, storage: st } };
  };
  $("#val").onclick = async () => { $("#out").textContent = JSON.stringify(await post("/validate/model", obj()), null, 2); };
  $("#go").onclick = async () => { try { await post("/models", obj()); location.hash = `models/${$("#n").value}`; } catch (e) { showErr(e); } };
}
function ModelImport() {
  page(`<h2>Import from Hugging Face</h2><p class="muted">Searches the local hub cache and models root (the console runs offline).</p>
    <div class="row"><input id="q" size="40" placeholder="search, e.g. llama"><button class="btn" id="s">search</button></div><div id="res"></div>`);
  $("#s").onclick = async () => {
    try {
      const { models } = await j(`/huggingface/models/search?q=${enc($("#q").value)}`);
      $("#res").innerHTML = table([["model", (m) => esc(m.id || m.modelId)], ["task", (m) => esc(m.pipeline_tag || "")],
        ["", (m) => `<button class="btn sec" data-id="${esc(m.id || m.modelId)}">import</button>`]], models);
      $$("#res button[data-id]").forEach((b) => b.onclick = async () => {
        const id = b.dataset.id;
        const info = await j(`/huggingface/models/${id}/info`).catch(() => ({}));
        const name = id.split("/").pop().toLowerCase().replace(/[^a-z0-9-]/g, "-");
        try {
          await post("/models", { metadata: { name }, spec: { vendor: id.split("/")[0], modelFormat: { name: "safetensors" },
            modelArchitecture: info.architecture || undefined, storage: { storageUri: `hf://${id}` } } });
          location.hash = `models/${name}`;
        } catch (e) { showErr(e, "#res"); }
      });
    } catch (e) { showErr(e, "#res"); }
  };
}
function editor(kindPath, back) {
  return async (name, ns) => {
    const q = ns ? `?namespace=${enc(ns)}` : "";
    const obj = await j(`/${kindPath}/${enc(name)}${q}`);
    page(`<h2>Edit ${esc(kindPath)}/${esc(name)}</h2><p class="muted">JSON or YAML; saved through the admission chain.</p>${jsonEditor(obj)}
      <div class="row"><button class="btn" id="save">save</button><a class="btn sec" href="#${back(name, ns)}">cancel</a></div>`);
    $("#save").onclick = async () => {
      try { await put(`/${kindPath}/${enc(name)}${q}`, $("#ed").value, "application/yaml"); location.hash = back(name, ns); } catch (e) { showErr(e); }
    };
  };
}

// ---------------------------------------------------------------- runtimes
async function RuntimeList() {
  const { items } = await j("/runtimes");
  page(`<h2>Cluster serving runtimes (${items.length})</h2><div class="row">${filterBox("rf")}<a class="btn" href="#runtimes/new">new runtime</a></div>` +
    table([["name", (r) => esc(r.metadata.name)],
      ["formats", (r) => esc((r.spec?.supportedModelFormats || []).map((f) => (f.modelFormat?.name || f.name) + (f.modelArchitecture ? "/" + f.modelArchitecture : "") + (f.quantization ? "/" + f.quantization : "")).join(", "))],
      ["size", (r) => esc(r.spec?.modelSizeRange ? `${r.spec.modelSizeRange.min}–${r.spec.modelSizeRange.max}` : "")],
      ["mode", (r) => esc(r.spec?.decoderConfig ? "PD" : r.spec?.engineConfig?.leader ? "multi-node" : "single")],
      ["state", (r) => r.spec?.disabled ? `<span class="warn">disabled</span>` : `<span class="ok">enabled</span>`]], items, (r) => `runtimes/${r.metadata.name}`));
  applyFilter("rf");
}
async function RuntimeDetail(name) {
  const r = await j(`/runtimes/${enc(name)}`);
  const runner = r.spec?.engineConfig?.runner || r.spec?.engineConfig?.leader?.runner || {};
  page(`<h2>${esc(name)}</h2><div class="row"><a class="btn sec" href="#runtimes/${enc(name)}/edit">edit</a>
      <a class="btn sec" href="#runtimes/${enc(name)}/clone">clone</a><button class="btn" id="del">delete</button></div>` +
    kv([["image", esc(runner.image)], ["command", `<code>${esc([...(runner.command || []), ...(runner.args || [])].join(" "))}</code>`],
      ["GPUs per pod", esc(runner.resources?.limits?.["amd.com/gpu"] ?? "")], ["router", esc(r.spec?.routerConfig ? "yes" : "no")],
      ["decoder (PD)", esc(r.spec?.decoderConfig ? "yes" : "no")], ["workers", esc(r.spec?.engineConfig?.worker?.size ?? "")],
      ["accelerators", esc((r.spec?.acceleratorRequirements?.acceleratorClasses || []).join(", "))]]) +
    `<h3>Check a model against this runtime</h3><div class="row"><input id="mm" placeholder="model name"><button class="btn" id="chk">check</button></div><pre id="cres"></pre>
     <h3>Object</h3><pre>${esc(JSON.stringify(r, null, 2))}</pre>`);
  $("#chk").onclick = async () => { try { $("#cres").textContent = JSON.stringify(await j(`/runtimes/${enc(name)}/compatibility?model=${enc($("#mm").value)}`), null, 2); } catch (e) { showErr(e); } };
  $("#del").onclick = async () => { if (confirm(`delete ${name}?`)) { try { await del(`/runtimes/${enc(name)}`); location.hash = "runtimes"; } catch (e) { showErr(e); } } };
}
function RuntimeClone(name) {
  page(`<h2>Clone ${esc(name)}</h2><label>new name</label><input id="nn" size="40" value="${esc(name)}-copy">
    <p class="muted">The clone is created disabled (an identical enabled copy would tie its source's auto-select priority).</p>
    <button class="btn" id="go">clone</button>`);
  $("#go").onclick = async () => { try { await post(`/runtimes/${enc(name)}/clone`, { newName: $("#nn").value }); location.hash = `runtimes/${$("#nn").value}/edit`; } catch (e) { showErr(e); } };
}
function RuntimeNew() {
  page(`<h2>New cluster serving runtime</h2><p class="muted">Paste a ClusterServingRuntime (YAML or JSON), or fetch one from the runtime catalog by path.</p>
    <div class="row"><input id="path" size="50" placeholder="ome-amd/llama-3-8b-instruct-rt.yaml"><button class="btn sec" id="fetch">fetch</button></div>
    <textarea id="ed"></textarea><div class="row"><button class="btn sec" id="val">validate</button><button class="btn" id="go">create</button></div><pre id="out"></pre>`);
  $("#fetch").onclick = async () => { try { const r = await j(`/runtimes/fetch-yaml?path=${enc($("#path").value)}`); $("#ed").value = r.yaml || JSON.stringify(r.runtime || r, null, 2); } catch (e) { showErr(e); } };
  $("#val").onclick = async () => { try { $("#out").textContent = JSON.stringify(await post("/validate/yaml", $("#ed").value, "application/yaml"), null, 2); } catch (e) { showErr(e); } };
  $("#go").onclick = async () => { try { const r = await post("/runtimes", $("#ed").value, "application/yaml"); location.hash = `runtimes/${r.metadata.name}`; } catch (e) { showErr(e); } };
}

// ---------------------------------------------------------------- services
async function ServiceList() {
  const { items } = await j("/services");
  page(`<h2>Inference services (${items.length})</h2><div class="row">${filterBox("sf")}<a class="btn" href="#services/deploy">deploy</a></div>` +
    table([["namespace", (s) => esc(s.metadata.namespace)], ["name", (s) => esc(s.metadata.name)], ["model", (s) => esc(s.spec?.model?.name)],
      ["runtime", (s) => esc(s.spec?.runtime?.name || "(auto)")], ["components", (s) => Object.keys(s.status?.components || {}).map((c) => `<span class="pill">${esc(c)}</span>`).join("")],
      ["state", (s) => badge(ready(s))], ["url", (s) => esc(s.status?.url || "")]], items, (s) => `services/${s.metadata.namespace}/${s.metadata.name}`));
  applyFilter("sf");
}
async function ServiceDetail(ns, name) {
  const [s, st] = await Promise.all([j(`/services/${enc(name)}?namespace=${enc(ns)}`), j(`/services/${enc(name)}/status?namespace=${enc(ns)}`)]);
  const comps = Object.entries(s.status?.components || {});
  page(`<h2>${esc(ns)}/${esc(name)} ${badge(st.ready ? "Ready" : "NotReady")}</h2><div class="row">
      <a class="btn sec" href="#services/${enc(ns)}/${enc(name)}/edit">edit</a><button class="btn" id="del">delete</button></div>` +
    kv([["model", `<a href="#models/${enc(s.spec?.model?.name || "")}">${esc(s.spec?.model?.name)}</a>`],
      ["runtime", esc(s.spec?.runtime?.name || "(auto-selected)")], ["url", esc(st.url || "")]]) +
    `<h3>Components</h3>${table([["component", (c) => esc(c[0])], ["ready", (c) => badge(c[1].ready ?? c[1].latestReadyRevision ? "Ready" : "-")],
      ["url", (c) => esc(c[1].url || "")]], comps)}
     <h3>Conditions</h3>${table([["type", (c) => esc(c.type)], ["status", (c) => badge(c.status)], ["reason", (c) => esc(c.reason || "")],
      ["message", (c) => esc(c.message || "")]], s.status?.conditions || [])}<h3>Object</h3><pre>${esc(JSON.stringify(s, null, 2))}</pre>`);
  $("#del").onclick = async () => { if (confirm(`delete ${ns}/${name}?`)) { try { await del(`/services/${enc(name)}?namespace=${enc(ns)}`); location.hash = "services"; } catch (e) { showErr(e); } } };
}
async function ServiceDeploy(_a, _b, query) {
  const models = (await j("/models")).items;
  const pre = query.get("model") || "";
  page(`<h2>Deploy an inference service</h2>
    <div class="row"><span class="step on">1 model</span> → <span class="step" id="s2">2 runtime</span> → <span class="step" id="s3">3 scale</span></div>
    <label>model</label><select id="m"><option value="">—</option>${models.map((m) => `<option ${m.metadata.name === pre ? "selected" : ""}>${esc(m.metadata.name)}</option>`).join("")}</select>
    <div id="rt"></div>
    <label>namespace</label><input id="ns" value="default"><label>service name</label><input id="nm" size="40">
    <label>engine replicas (min / max)</label><input id="mn" value="1" size="4"> <input id="mx" value="1" size="4">
    <label><input type="checkbox" id="pd"> prefill/decode disaggregation (decoder component)</label>
    <div class="row"><button class="btn sec" id="val">validate</button><button class="btn" id="go">deploy</button></div><pre id="out"></pre>`);
  let runtime = "";
  const pickModel = async () => {
    const m = $("#m").value;
    if (!m) { $("#rt").innerHTML = ""; return; }
    $("#nm").value = $("#nm").value || m;
    $("#s2").classList.add("on");
    const c = await j(`/runtimes/compatible?model=${enc(m)}`).catch(() => ({ runtimes: [] }));
    $("#rt").innerHTML = `<label>runtime</label><select id="r"><option value="">(auto-select)</option>${(c.runtimes || []).map((r) =>
      `<option value="${esc(r.runtime)}">${esc(r.runtime)} — score ${esc(r.score)}</option>`).join("")}</select>`;
    $("#r").onchange = () => { runtime = $("#r").value; $("#s3").classList.add("on"); };
  };
  $("#m").onchange = pickModel;
  if (pre) pickModel();
  const obj = () => {
    const spec = { model: { name: $("#m").value }, engine: { minReplicas: +$("#mn").value, maxReplicas: +$("#mx").value } };
    if (runtime) spec.runtime = { name: runtime };
    if ($("#pd").checked) { spec.decoder = { minReplicas: 1, maxReplicas: 1 }; spec.router = { minReplicas: 1, maxReplicas: 1 }; }
    return { apiVersion: "ome.io/v1beta1", kind: "InferenceService", metadata: { name: $("#nm").value, namespace: $("#ns").value }, spec };
  };
  $("#val").onclick = async () => { $("#out").textContent = JSON.stringify(await post("/validate/yaml", JSON.stringify(obj()), "application/yaml"), null, 2); };
  $("#go").onclick = async () => { try { const o = obj(); await post(`/services?namespace=${enc(o.metadata.namespace)}`, o); location.hash = `services/${o.metadata.namespace}/${o.metadata.name}`; } catch (e) { showErr(e); } };
}

// ---------------------------------------------------------------- accelerators / benchmarks / validate
async function AcceleratorList() {
  const { items } = await j("/accelerators");
  page(`<h2>Accelerator classes (${items.length})</h2>` + table([["name", (a) => esc(a.metadata.name)], ["vendor", (a) => esc(a.spec?.vendor)],
    ["family / model", (a) => esc(`${a.spec?.family || ""} ${a.spec?.model || ""}`)], ["memory GB", (a) => esc(a.spec?.capabilities?.memoryGB)],
    ["nodes", (a) => esc(a.status?.availableNodes?.length ?? a.status?.nodes?.length ?? "")]], items, (a) => `accelerators/${a.metadata.name}`));
}
async function AcceleratorDetail(name) {
  const a = await j(`/accelerators/${enc(name)}`);
  page(`<h2>${esc(name)}</h2>` + kv(Object.entries(a.spec?.capabilities || {}).map(([k, v]) => [k, esc(typeof v === "object" ? JSON.stringify(v) : v)])) +
    `<h3>Discovery</h3><pre>${esc(JSON.stringify(a.spec?.discovery || {}, null, 2))}</pre><h3>Status</h3><pre>${esc(JSON.stringify(a.status || {}, null, 2))}</pre>`);
}
async function BenchmarkList() {
  const { items } = await j("/benchmarks");
  page(`<h2>Benchmark jobs (${items.length})</h2>` + table([["namespace/name", (b) => esc(`${b.metadata.namespace}/${b.metadata.name}`)],
    ["endpoint", (b) => esc(b.spec?.endpoint?.inferenceService?.name || b.spec?.endpoint?.endpoint?.url || "")], ["task", (b) => esc(b.spec?.task)],
    ["scenarios", (b) => (b.spec?.trafficScenarios || []).map((s) => `<span class="pill">${esc(s)}</span>`).join("")],
    ["concurrency", (b) => esc((b.spec?.numConcurrency || []).join(","))], ["state", (b) => badge(b.status?.state || ready(b))]],
    items, (b) => `benchmarks/${b.metadata.namespace}/${b.metadata.name}`) +
    `<h3>New benchmark job</h3><textarea id="ed">apiVersion: ome.io/v1beta1\nkind: BenchmarkJob\nmetadata:\n  name: bench\n  namespace: default\nspec:\n  endpoint:\n    inferenceService:\n      name: llama-3-8b-instruct\n      namespace: default\n  task: text-to-text\n  trafficScenarios: ["N(480,240)/(300,150)", "D(100,100)"]\n  numConcurrency: [1, 8, 64, 256]\n  maxTimePerIteration: 15\n  maxRequestsPerIteration: 100\n  outputLocation:\n    storageUri: local:///tmp/ome-bench-results\n</textarea>
     <div class="row"><button class="btn" id="go">create</button></div>`);
  $("#go").onclick = async () => { try { await post("/benchmarks", $("#ed").value, "application/yaml"); BenchmarkList(); } catch (e) { showErr(e); } };
}
async function BenchmarkDetail(ns, name) {
  const b = await j(`/benchmarks/${enc(name)}?namespace=${enc(ns)}`);
  page(`<h2>${esc(ns)}/${esc(name)} ${badge(b.status?.state || ready(b))}</h2>` +
    kv([["task", esc(b.spec?.task)], ["scenarios", esc((b.spec?.trafficScenarios || []).join(", "))], ["concurrency", esc((b.spec?.numConcurrency || []).join(", "))],
      ["results", esc(b.spec?.outputLocation?.storageUri || "")], ["started", esc(b.status?.startTime || "")], ["finished", esc(b.status?.completionTime || "")]]) +
    `<h3>Status</h3><pre>${esc(JSON.stringify(b.status || {}, null, 2))}</pre>`);
}
function Validate() {
  page(`<h2>Validate manifests</h2><p class="muted">Runs the manager's admission chain (defaulting + validation) without persisting.</p>
    <textarea id="ed">apiVersion: ome.io/v1beta1\nkind: InferenceService\nmetadata:\n  name: llama3-8b\n  namespace: default\nspec:\n  model:\n    name: llama-3-8b-instruct\n</textarea>
    <div class="row"><button class="btn" id="val">validate</button></div><pre id="out"></pre>`);
  $("#val").onclick = async () => { $("#out").textContent = JSON.stringify(await post("/validate/yaml", $("#ed").value, "application/yaml"), null, 2); };
}

// ---------------------------------------------------------------- router
const ROUTES = [
  [/^$|^dashboard$/, Dashboard, "dashboard"],
  [/^models$/, ModelList, "models"], [/^models\/new$/, ModelNew, "models"], [/^models\/import$/, ModelImport, "models"],
  [/^models\/([^/]+)\/edit$/, editor("models", (n) => `models/${n}`), "models"], [/^models\/([^/]+)$/, ModelDetail, "models"],
  [/^runtimes$/, RuntimeList, "runtimes"], [/^runtimes\/new$/, RuntimeNew, "runtimes"],
  [/^runtimes\/([^/]+)\/clone$/, RuntimeClone, "runtimes"], [/^runtimes\/([^/]+)\/edit$/, editor("runtimes", (n) => `runtimes/${n}`), "runtimes"],
  [/^runtimes\/([^/]+)$/, RuntimeDetail, "runtimes"],
  [/^services$/, ServiceList, "services"], [/^services\/deploy$/, ServiceDeploy, "services"],
  [/^services\/([^/]+)\/([^/]+)\/edit$/, (ns, n) => editor("services", (n2, ns2) => `services/${ns2}/${n2}`)(n, ns), "services"],
  [/^services\/([^/]+)\/([^/]+)$/, ServiceDetail, "services"],
  [/^accelerators$/, AcceleratorList, "accelerators"], [/^accelerators\/([^/]+)$/, AcceleratorDetail, "accelerators"],
  [/^benchmarks$/, BenchmarkList, "benchmarks"], [/^benchmarks\/([^/]+)\/([^/]+)$/, BenchmarkDetail, "benchmarks"],
  [/^validate$/, Validate, "validate"],
];
const NAV = ["dashboard", "models", "runtimes", "services", "accelerators", "benchmarks", "validate"];
function route() {
  const [path, qs] = location.hash.slice(1).split("?");
  const query = new URLSearchParams(qs || "");
  for (const [re, fn, tab] of ROUTES) {
    const m = path.match(re);
    if (!m) continue;
    $("#nav").innerHTML = NAV.map((t) => `<a href="#${t}" class="${t === tab ? "on" : ""}">${t}</a>`).join("");
    Promise.resolve(fn(...m.slice(1).map(decodeURIComponent), query)).catch((e) => page(`<div class="err">${esc(e.message)}</div>`));
    return;
  }
  location.hash = "dashboard";
}
window.onhashchange = route;
fetch("health").then((r) => r.json()).then((h) => { $("#health").textContent = `api ${h.status}`; }).catch(() => { $("#health").textContent = "api unreachable"; });
const es = new EventSource(`${API}/events`);
es.addEventListener("connected", () => { $("#conn").textContent = "connected"; });
for (const t of ["add", "update", "delete"]) es.addEventListener(t, (ev) => {
  const m = JSON.parse(ev.data);
  $("#feed").insertAdjacentHTML("afterbegin", `<div><span class="${t === "delete" ? "bad" : t === "add" ? "ok" : "muted"}">${t}</span> ${esc(m.resource)} ${esc(m.namespace ? m.namespace + "/" : "")}${esc(m.name)}</div>`);
  const cur = location.hash.slice(1).split("/")[0] || "dashboard";
  if (cur === m.resource && !location.hash.includes("/edit") && !location.hash.includes("/new") && !location.hash.includes("deploy")) route();
});
route();
