// ome-amd web console — hash-routed single-page app over the console REST API (api/v1).
// Views follow the reference Next.js dashboard (web-console/frontend/src/app/(dashboard)/*):
// dashboard (StatsGrid), models (list / detail / new / import / edit, cluster and namespaced),
// runtimes (list / detail / new / import / clone / edit), services (list / detail / deploy),
// accelerators, benchmarks and manifest validation; tables sort, filter, bulk-delete and export
// (components/layout/ResourceTable, ui/DataTable + BulkActionDropdown, lib/utils/export.ts); a
// namespace selector scopes namespaced kinds (lib/hooks/useNamespaces.ts); server-sent events keep
// lists live (lib/hooks/useServerEvents.ts).  Pure helpers: lib.js; form widgets: forms.js.
"use strict";
const API = "api/v1";
const { esc, toYaml, toCsv, sortRows, ago, fmtBytes } = OME;
const F = OMEForms;
const $ = (s, el = document) => el.querySelector(s);
const $$ = (s, el = document) => [...el.querySelectorAll(s)];
const enc = encodeURIComponent;

async function j(path, opt) {
  const r = await fetch(`${API}${path}`, opt);
  const body = await r.json().catch(() => ({}));
  if (!r.ok) {
    const d = body.detail;
    throw new Error(typeof d === "object" ? [d.error, Array.isArray(d.details) ? d.details.join("; ") : d.details].filter(Boolean).join(": ") || JSON.stringify(d)
                                          : (d || JSON.stringify(body)));
  }
  return body;
}
const send = (method, path, obj, type = "application/json") =>
  j(path, { method, headers: { "Content-Type": type }, body: typeof obj === "string" ? obj : JSON.stringify(obj) });
const post = (p, o, t) => send("POST", p, o, t);
const put = (p, o, t) => send("PUT", p, o, t);
const del = (p) => j(p, { method: "DELETE" });

// ---------------------------------------------------------------- namespace scope
const NS = {
  get: () => localStorage.getItem("ome.ns") || "all",
  set: (v) => localStorage.setItem("ome.ns", v),
  query: (sep = "?") => (NS.get() === "all" ? "" : `${sep}namespace=${enc(NS.get())}`),
};
async function loadNamespaces() {
  const { namespaces } = await j("/namespaces").catch(() => ({ namespaces: ["default"] }));
  const cur = NS.get();
  $("#nssel").innerHTML = ["all", ...namespaces].map((n) => `<option ${n === cur ? "selected" : ""}>${esc(n)}</option>`).join("");
  $("#nssel").onchange = (e) => { NS.set(e.target.value); route(); };
  return namespaces;
}

// ---------------------------------------------------------------- view helpers
function ready(o) {
  const st = o.status || {};
  if (st.state) return st.state;
  const c = (st.conditions || []).find((c) => c.type === "Ready");
  return c ? (c.status === "True" ? "Ready" : c.status === "False" ? "NotReady" : "Unknown") : "-";
}
function badge(s) {
  const cls = ["Ready", "True", "Completed", "Succeeded", "enabled"].includes(s) ? "ok" : ["Failed", "False", "NotReady"].includes(s) ? "bad" : "warn";
  return `<span class="badge ${cls}">${esc(s)}</span>`;
}
const pills = (xs) => (xs || []).map((c) => `<span class="pill">${esc(c)}</span>`).join("");
function kv(pairs) { return `<div class="kv">${pairs.filter((p) => p[1] !== undefined).map(([k, v]) => `<div>${esc(k)}</div><div>${v}</div>`).join("")}</div>`; }
function page(html) { $("#page").innerHTML = html; }
function showErr(e, where = "#page") { $(where).insertAdjacentHTML("afterbegin", `<div class="err">${esc(e.message || e)}</div>`); }
function copyBtn(text) { return `<button class="btn sec copy" type="button" data-copy="${esc(text)}">copy</button>`; }
function wireCopy(el = document) { $$("[data-copy]", el).forEach((b) => { b.onclick = () => navigator.clipboard && navigator.clipboard.writeText(b.dataset.copy); }); }
function download(name, text, type) {
  const a = document.createElement("a");
  a.href = URL.createObjectURL(new Blob([text], { type }));
  a.download = name;
  a.click();
  setTimeout(() => URL.revokeObjectURL(a.href), 1000);
}
function cleanForEdit(obj) {
  const o = JSON.parse(JSON.stringify(obj));
  if (o.metadata) for (const k of ["uid", "creationTimestamp", "generation", "managedFields", "resourceVersion"]) delete o.metadata[k];
  delete o.status;
  return o;
}

// Sortable / filterable / selectable table with bulk delete and CSV / JSON / YAML export.
// cols: [[header, render(row) -> html, sortKey(row)?, exportValue(row)?], ...]
function dataTable(el, { cols, rows, href, name, onDelete, rowId }) {
  let sortCol = -1, dir = 1, filter = "";
  const selected = new Set();
  const id = rowId || ((r) => `${r.metadata.namespace ? r.metadata.namespace + "/" : ""}${r.metadata.name}`);
  const draw = () => {
    let rs = rows.filter((r) => !filter || JSON.stringify([r.metadata, r.spec]).toLowerCase().includes(filter));
    if (sortCol >= 0) { const c = cols[sortCol]; rs = sortRows(rs, c[2] || ((r) => c[1](r).replace(/<[^>]*>/g, "")), dir); }
    const body = rs.map((r) => `<tr class="${href ? "click" : ""}" data-id="${esc(id(r))}" ${href ? `data-href="${esc(href(r))}"` : ""}>
        ${onDelete ? `<td class="cb"><input type="checkbox" ${selected.has(id(r)) ? "checked" : ""}></td>` : ""}
        ${cols.map((c) => `<td>${c[1](r)}</td>`).join("")}</tr>`).join("");
    el.innerHTML = `<div class="row tools"><input class="filter" placeholder="filter…" size="24" value="${esc(filter)}">
        <span class="muted">${rs.length} of ${rows.length}</span>
        ${onDelete ? `<button class="btn sec" data-bulk ${selected.size ? "" : "disabled"}>delete selected (${selected.size})</button>` : ""}
        <span class="spacer"></span><button class="btn sec" data-exp="csv">CSV</button><button class="btn sec" data-exp="json">JSON</button>
        <button class="btn sec" data-exp="yaml">YAML</button></div>` +
      (rows.length ? `<table class="dt"><tr>${onDelete ? `<th class="cb"><input type="checkbox" data-all></th>` : ""}${cols.map((c, i) =>
        `<th class="sortable" data-col="${i}">${esc(c[0])}${i === sortCol ? (dir > 0 ? " ▲" : " ▼") : ""}</th>`).join("")}</tr>${body}</table>` : `<p class="muted">none</p>`);
    const f = $(".filter", el);
    f.oninput = () => { filter = f.value.toLowerCase(); const pos = f.selectionStart; draw(); const g = $(".filter", el); g.focus(); g.setSelectionRange(pos, pos); };
    $$("th.sortable", el).forEach((th) => { th.onclick = () => { const c = +th.dataset.col; dir = c === sortCol ? -dir : 1; sortCol = c; draw(); }; });
    $$("tr[data-href] td:not(.cb)", el).forEach((td) => { td.onclick = () => { location.hash = td.parentElement.dataset.href; }; });
    $$("td.cb input", el).forEach((cb) => { cb.onchange = () => { const k = cb.closest("tr").dataset.id; cb.checked ? selected.add(k) : selected.delete(k); draw(); }; });
    const all = $("[data-all]", el);
    if (all) all.onchange = () => { rs.forEach((r) => (all.checked ? selected.add(id(r)) : selected.delete(id(r)))); draw(); };
    const bulk = $("[data-bulk]", el);
    if (bulk) bulk.onclick = async () => {
      const victims = rows.filter((r) => selected.has(id(r)));
      if (!confirm(`delete ${victims.length} object(s)?\n${victims.map(id).join("\n")}`)) return;
      const errs = [];
      for (const r of victims) { try { await onDelete(r); selected.delete(id(r)); } catch (e) { errs.push(`${id(r)}: ${e.message}`); } }
      rows = rows.filter((r) => !victims.includes(r) || selected.has(id(r)));
      draw();
      if (errs.length) showErr(new Error(errs.join("\n")), `#${el.id}`);
    };
    $$("[data-exp]", el).forEach((b) => { b.onclick = () => {
      const fmt = b.dataset.exp, stamp = new Date().toISOString().slice(0, 10);
      if (fmt === "csv") download(`${name}-${stamp}.csv`, toCsv(cols.map((c) => [c[0], c[3] || ((r) => c[1](r).replace(/<[^>]*>/g, ""))]), rs), "text/csv");
      else if (fmt === "json") download(`${name}-${stamp}.json`, JSON.stringify(rs, null, 2), "application/json");
      else download(`${name}-${stamp}.yaml`, rs.map((r) => toYaml(cleanForEdit(r))).join("\n---\n") + "\n", "application/yaml");
    }; });
  };
  draw();
}

// a structured form next to a live YAML preview, with validate + submit
function formPage({ title, intro, body, build, errors, submit, validatePath }) {
  page(`<h2>${esc(title)}</h2>${intro ? `<p class="muted">${intro}</p>` : ""}<div class="formgrid"><div id="form">${body}</div>
      <div><h3>manifest</h3><pre id="preview"></pre><ul id="ferrs" class="bad"></ul></div></div>
      <div class="row"><button class="btn sec" id="val">server-side validate</button><button class="btn" id="go">create</button></div><pre id="out"></pre>`);
  const refresh = () => {
    try {
      $("#preview").textContent = toYaml(build());
      $("#ferrs").innerHTML = (errors ? errors() : []).map((e) => `<li>${esc(e)}</li>`).join("");
    } catch (e) { $("#preview").textContent = String(e); }
  };
  $("#form").addEventListener("input", refresh);
  $("#form").addEventListener("change", refresh);
  $("#val").onclick = async () => {
    try { $("#out").textContent = JSON.stringify(await post(validatePath || "/validate/yaml", toYaml(build()), "application/yaml"), null, 2); } catch (e) { showErr(e); }
  };
  $("#go").onclick = async () => {
    const errs = errors ? errors() : [];
    if (errs.length) { showErr(new Error(errs.join("\n"))); return; }
    try { await submit(build()); } catch (e) { showErr(e); }
  };
  return refresh;
}

// ---------------------------------------------------------------- dashboard
async function Dashboard() {
  const [sum, svcs, models, rts] = await Promise.all([j("/summary"), j(`/services${NS.query()}`), j("/models"), j("/runtimes")]);
  const card = (label, val, href, sub) => `<a class="card" href="#${href}"><b>${val}</b><span>${label}</span>${sub ? `<i>${sub}</i>` : ""}</a>`;
  const frac = (c) => `${c.ready ?? 0}/${c.total ?? 0}`;
  const byState = (xs) => xs.reduce((m, x) => { const s = ready(x); m[s] = (m[s] || 0) + 1; return m; }, {});
  const stateLine = (xs) => Object.entries(byState(xs)).map(([s, n]) => `${badge(s)} ${n}`).join(" ");
  const enabled = rts.items.filter((r) => !(r.spec || {}).disabled).length;
  page(`<h2>Dashboard</h2><div class="cards">
      ${card("base models ready", frac(sum.models), "models", stateLine(models.items))}
      ${card("services ready", frac(sum.services), "services", stateLine(svcs.items))}
      ${card("serving runtimes", sum.runtimes.total, "runtimes", `${enabled} enabled`)}
      ${card("accelerator classes", sum.accelerators.total, "accelerators")}
      ${card("benchmark jobs", sum.benchmarks.total, "benchmarks")}
      <div class="card"><b>${sum.nodes}</b><span>nodes</span></div></div>
    <h3>Inference services${NS.get() === "all" ? "" : ` in ${esc(NS.get())}`}</h3><div id="t1"></div>
    <h3>Models not ready</h3><div id="t2"></div>`);
  dataTable($("#t1"), { name: "services", rows: svcs.items, href: (s) => `services/${s.metadata.namespace}/${s.metadata.name}`,
    cols: [["namespace/name", (s) => esc(`${s.metadata.namespace}/${s.metadata.name}`)], ["model", (s) => esc(s.spec?.model?.name)],
      ["state", (s) => badge(ready(s)), ready], ["url", (s) => esc(s.status?.url || "")]] });
  dataTable($("#t2"), { name: "models-not-ready", rows: models.items.filter((m) => ready(m) !== "Ready"), href: (m) => `models/${m.metadata.name}`,
    cols: [["name", (m) => esc(m.metadata.name)], ["state", (m) => badge(ready(m)), ready], ["storage", (m) => esc(m.spec?.storage?.storageUri)]] });
}

// ---------------------------------------------------------------- models
const modelCols = [
  ["name", (m) => esc(m.metadata.name), (m) => m.metadata.name],
  ["vendor", (m) => esc(m.spec?.vendor), (m) => m.spec?.vendor],
  ["architecture", (m) => esc(m.spec?.modelArchitecture), (m) => m.spec?.modelArchitecture],
  ["size", (m) => esc(m.spec?.modelParameterSize), (m) => m.spec?.modelParameterSize],
  ["format", (m) => esc(m.spec?.modelFormat?.name), (m) => m.spec?.modelFormat?.name],
  ["quant", (m) => esc(m.spec?.quantization || ""), (m) => m.spec?.quantization],
  ["capabilities", (m) => pills(m.spec?.modelCapabilities), (m) => (m.spec?.modelCapabilities || []).join(","), (m) => (m.spec?.modelCapabilities || []).join(" ")],
  ["state", (m) => badge(ready(m)), ready, ready],
  ["nodes", (m) => esc((m.status?.nodesReady || []).length), (m) => (m.status?.nodesReady || []).length],
  ["age", (m) => esc(ago(m.metadata.creationTimestamp)), (m) => -Date.parse(m.metadata.creationTimestamp || 0)],
];
async function ModelList() {
  const scope = NS.get();
  const cluster = await j("/models");
  const nsList = scope === "all" ? (await j("/namespaces")).namespaces : [scope];
  const nsModels = (await Promise.all(nsList.map((n) => j(`/namespaces/${enc(n)}/models`).catch(() => ({ items: [] }))))).flatMap((r) => r.items);
  page(`<h2>Base models</h2><div class="row"><a class="btn" href="#models/new">new model</a><a class="btn sec" href="#models/import">import from Hugging Face</a></div>
    <h3>Cluster base models (${cluster.items.length})</h3><div id="tc"></div>
    <h3>Namespaced base models (${nsModels.length}${scope === "all" ? "" : ` in ${esc(scope)}`})</h3><div id="tn"></div>`);
  dataTable($("#tc"), { name: "clusterbasemodels", rows: cluster.items, cols: modelCols, href: (m) => `models/${m.metadata.name}`,
    onDelete: (m) => del(`/models/${enc(m.metadata.name)}`) });
  dataTable($("#tn"), { name: "basemodels", rows: nsModels, cols: [["namespace", (m) => esc(m.metadata.namespace), (m) => m.metadata.namespace], ...modelCols],
    href: (m) => `models/ns/${m.metadata.namespace}/${m.metadata.name}`,
    onDelete: (m) => del(`/namespaces/${enc(m.metadata.namespace)}/models/${enc(m.metadata.name)}`) });
}
async function ModelDetail(a, b) {
  const ns = b === undefined ? null : a, name = b === undefined ? a : b;
  const base = ns ? `/namespaces/${enc(ns)}/models/${enc(name)}` : `/models/${enc(name)}`;
  const m = await j(base);
  const [prog, ev] = ns ? [{ progress: [] }, { events: [] }] : await Promise.all([j(`${base}/progress`), j(`${base}/events`)]);
  const rq = `model=${enc(name)}${ns ? `&namespace=${enc(ns)}` : ""}`;
  const rec = await j(`/runtimes/recommend?${rq}`).catch((e) => ({ error: e.message }));
  const compat = await j(`/runtimes/compatible?${rq}`).catch(() => ({ runtimes: [] }));
  const sp = m.spec || {}, st = m.status || {};
  const bars = (prog.progress || []).map((p) => `<div>${esc(p.node)} · ${esc(p.phase)} ${Number(p.percentage || 0).toFixed(1)}%
      <span class="muted">${fmtBytes(p.completedBytes)} / ${fmtBytes(p.totalBytes)} · ${fmtBytes(p.bytesPerSecond)}/s</span>
      <div class="bar"><i style="width:${Number(p.percentage || 0)}%"></i></div></div>`).join("") || `<p class="muted">no download in progress</p>`;
  const editHref = ns ? `models/ns/${enc(ns)}/${enc(name)}/edit` : `models/${enc(name)}/edit`;
  page(`<h2>${esc(ns ? `${ns}/${name}` : name)} ${badge(ready(m))}</h2><div class="row"><a class="btn sec" href="#${editHref}">edit</a>
      <a class="btn sec" href="#services/deploy?model=${enc(name)}${ns ? `&namespace=${enc(ns)}` : ""}">deploy</a><button class="btn" id="del">delete</button></div>
    <div class="grid2"><div>${kv([["kind", esc(m.kind)], ["storage", `<code>${esc(sp.storage?.storageUri)}</code> ${copyBtn(sp.storage?.storageUri || "")}`],
      ["path on nodes", esc(sp.storage?.path)], ["storage key", esc(sp.storage?.key)],
      ["node selector", esc(JSON.stringify(sp.storage?.nodeSelector || {}))], ["architecture", esc(sp.modelArchitecture)],
      ["parameters", esc(sp.modelParameterSize)], ["format", esc(`${sp.modelFormat?.name || ""} ${sp.modelFormat?.version || ""}`)],
      ["framework", esc(`${sp.modelFramework?.name || ""} ${sp.modelFramework?.version || ""}`)], ["quantization", esc(sp.quantization || "")],
      ["capabilities", pills(sp.modelCapabilities)], ["max tokens", esc(sp.maxTokens || "")]])}</div>
      <div>${kv([["state", badge(ready(m))], ["lifecycle", esc(st.lifecycle || "")], ["nodes ready", pills(st.nodesReady)], ["nodes failed", pills(st.nodesFailed)],
      ["recommended runtime", rec.runtime ? `<a href="#runtimes/${enc(rec.runtime)}">${esc(rec.runtime)}</a> (score ${esc(rec.score)})` : esc(rec.error || "-")],
      ["created", esc(m.metadata.creationTimestamp || "")]])}</div></div>
    <h3>Download progress</h3>${bars}<h3>Compatible runtimes</h3><div id="tr"></div>
    <h3>Events</h3>${(ev.events || []).map((e) => `<div class="muted">${esc(e.lastTimestamp || "")} ${esc(e.reason)}: ${esc(e.message)}</div>`).join("") || "<p class='muted'>none</p>"}
    <details class="sec"><summary>Object (YAML)</summary><pre>${esc(toYaml(m))}</pre></details>`);
  dataTable($("#tr"), { name: "compatible-runtimes", rows: compat.runtimes || [], rowId: (r) => r.runtime, href: (r) => `runtimes/${r.runtime}`,
    cols: [["runtime", (r) => esc(r.runtime), (r) => r.runtime], ["score", (r) => esc(r.score), (r) => r.score], ["why", (r) => esc((r.reasons || []).join("; "))]] });
  wireCopy();
  $("#del").onclick = async () => { if (confirm(`delete ${name}?`)) { try { await del(base); location.hash = "models"; } catch (e) { showErr(e); } } };
}
const CAPS = ["TEXT_GENERATION", "CHAT", "EMBEDDING", "VISION", "IMAGE_GENERATION", "AUDIO", "RERANK", "TEXT_TO_IMAGE", "IMAGE_TEXT_TO_TEXT"];
function modelFormBody(pre = {}) {
  const sp = pre.spec || {};
  return `<div id="mb" class="grid2">
      ${F.field("name", F.inp("name", pre.metadata?.name || "", "my-model", 32))}
      ${F.field("scope", F.sel("namespace", [["", "cluster (ClusterBaseModel)"], ...(window.__namespaces || ["default"]).map((n) => [n, `namespace ${n} (BaseModel)`])], pre.metadata?.namespace || ""))}
      ${F.field("vendor", F.inp("vendor", sp.vendor || "", "e.g., meta, openai", 20))}
      ${F.field("display name", F.inp("displayName", sp.displayName || "", "", 24))}
      ${F.field("architecture", F.inp("architecture", sp.modelArchitecture || "", "LlamaForCausalLM", 24))}
      ${F.field("parameter size", F.inp("parameterSize", sp.modelParameterSize || "", "e.g., 7B, 13B, 70B", 10))}
      ${F.field("format / version", F.sel("formatName", ["safetensors", "pytorch", "gguf", "onnx", "tensorrt"], sp.modelFormat?.name || "safetensors") + " " + F.inp("formatVersion", sp.modelFormat?.version || "", "1.0.0", 6))}
      ${F.field("framework / version", F.inp("frameworkName", sp.modelFramework?.name || "", "transformers", 12) + " " + F.inp("frameworkVersion", sp.modelFramework?.version || "", "4.46.0", 6))}
      ${F.field("quantization", F.sel("quantization", F.QUANT, sp.quantization || ""))}
      ${F.field("max tokens", F.inp("maxTokens", sp.maxTokens || "", "131072", 8))}
      ${F.field("local path on nodes", F.inp("path", sp.storage?.path || "", "/raid/models/meta-llama/llama-3.1-8b-instruct", 36))}
      ${F.field("storage key (Secret)", F.inp("storageKey", sp.storage?.key || "", "", 20))}
      ${F.field("Hugging Face token", F.inp("huggingFaceToken", "", "hf_...", 24, "password"), "stored as a Secret the model agent reads")}
      ${F.chk("disabled", sp.disabled, "disabled")}</div>
    <label>capabilities</label><div id="caps" class="row">${CAPS.map((c) => F.chk(`cap:${c}`, (sp.modelCapabilities || []).includes(c), c)).join("")}</div>
    ${F.section("storage", `<div id="stor"></div><label>node selector</label><div id="nsel"></div><label>storage parameters</label><div id="sparams"></div>`)}
    ${F.section("labels", `<div id="labels"></div>`, false)}`;
}
function modelFormWire(pre = {}) {
  const sp = pre.spec || {};
  const stor = F.StorageBuilder($("#stor"), sp.storage?.storageUri || "");
  const nsel = F.KVEditor($("#nsel"), Object.entries(sp.storage?.nodeSelector || {}), { addLabel: "selector" });
  const sparams = F.KVEditor($("#sparams"), Object.entries(sp.storage?.parameters || {}), { addLabel: "parameter" });
  const labels = F.KVEditor($("#labels"), Object.entries(pre.metadata?.labels || {}), { addLabel: "label" });
  return () => {
    const b = F.read($("#mb"));
    const caps = Object.entries(F.read($("#caps"))).filter(([, v]) => v).map(([k]) => k.slice(4));
    return { ...b, capabilities: caps, storageUri: stor.value(), nodeSelector: nsel.value(), parameters: sparams.value(), labels: labels.value() };
  };
}
function ModelNew() {
  let state = () => ({});
  const refresh = formPage({ title: "New base model", intro: "Structured form (reference models/new); the manifest on the right is what gets created.",
    body: modelFormBody(), build: () => OME.buildModel(state()), errors: () => OME.modelErrors(state()), validatePath: "/validate/yaml",
    submit: async (obj) => {
      if (obj.kind === "BaseModel") { const ns = obj.metadata.namespace; await post(`/namespaces/${enc(ns)}/models`, obj); location.hash = `models/ns/${ns}/${obj.metadata.name}`; }
      else { await post("/models", obj); location.hash = `models/${obj.metadata.name}`; }
    } });
  state = modelFormWire();
  refresh();
}
function ModelImport() {
  page(`<h2>Import from Hugging Face</h2><p class="muted">Searches the local hub cache and models root (the console runs offline); the
    model's config.json fills architecture, size and format.</p>
    <div class="row"><input id="q" size="40" placeholder="Search for models (e.g., meta-llama/Llama-2-7b)"><button class="btn" id="s">search</button></div>
    <div class="row">${F.field("scope", `<select id="scope"><option value="">cluster</option>${(window.__namespaces || []).map((n) => `<option>${esc(n)}</option>`).join("")}</select>`)}
      ${F.field("Hugging Face token (optional)", `<input id="tok" type="password" size="24" placeholder="hf_...">`)}</div><div id="res"></div>`);
  $("#s").onclick = async () => {
    try {
      const { models } = await j(`/huggingface/models/search?q=${enc($("#q").value)}`);
      const rows = (models || []).map((m) => ({ ...m, metadata: { name: m.id || m.modelId } }));
      $("#res").innerHTML = `<div id="rt"></div>`;
      dataTable($("#rt"), { name: "hf-search", rows, rowId: (m) => m.metadata.name,
        cols: [["model", (m) => esc(m.metadata.name), (m) => m.metadata.name], ["task", (m) => esc(m.pipeline_tag || "")],
          ["downloads", (m) => esc(m.downloads ?? ""), (m) => m.downloads || 0], ["", (m) => `<button class="btn sec" data-id="${esc(m.metadata.name)}">import</button>`]] });
      $$("#res button[data-id]").forEach((b) => b.onclick = async (ev) => {
        ev.stopPropagation();
        const id = b.dataset.id, ns = $("#scope").value;
        const info = await j(`/huggingface/models/${id}/info`).catch(() => ({}));
        const name = id.split("/").pop().toLowerCase().replace(/[^a-z0-9-]/g, "-").replace(/^-+|-+$/g, "");
        const obj = OME.buildModel({ name, namespace: ns, vendor: id.split("/")[0], formatName: info.format || "safetensors",
          architecture: info.architecture, parameterSize: info.parameterSize || info.modelParameterSize, storageUri: `hf://${id}`,
          huggingFaceToken: $("#tok").value, capabilities: info.capabilities });
        try {
          if (ns) { await post(`/namespaces/${enc(ns)}/models`, obj); location.hash = `models/ns/${ns}/${name}`; }
          else { await post("/models", obj); location.hash = `models/${name}`; }
        } catch (e) { showErr(e, "#res"); }
      });
    } catch (e) { showErr(e, "#res"); }
  };
}
// YAML/JSON editor for any object, saved through the admission chain
function editor(pathOf, back) {
  return async (...args) => {
    const path = pathOf(...args);
    const obj = await j(path);
    page(`<h2>Edit ${esc(obj.kind)} ${esc(obj.metadata?.namespace ? obj.metadata.namespace + "/" : "")}${esc(obj.metadata?.name)}</h2>
      <p class="muted">YAML or JSON; saved through the admission chain (defaulting + validation).</p>
      <textarea id="ed">${esc(toYaml(cleanForEdit(obj)))}</textarea>
      <div class="row"><button class="btn" id="save">save</button><button class="btn sec" id="val">validate</button><a class="btn sec" href="#${back(...args)}">cancel</a></div><pre id="out"></pre>`);
    $("#val").onclick = async () => { try { $("#out").textContent = JSON.stringify(await post("/validate/yaml", $("#ed").value, "application/yaml"), null, 2); } catch (e) { showErr(e); } };
    $("#save").onclick = async () => { try { await put(path, $("#ed").value, "application/yaml"); location.hash = back(...args); } catch (e) { showErr(e); } };
  };
}

// ---------------------------------------------------------------- runtimes
const fmtList = (r) => (r.spec?.supportedModelFormats || []).map((f) => (f.modelFormat?.name || f.name) + (f.modelArchitecture ? "/" + f.modelArchitecture : "") + (f.quantization ? "/" + f.quantization : ""));
const rtMode = (r) => (r.spec?.decoderConfig ? "PD" : r.spec?.engineConfig?.leader ? "multi-node" : "single");
async function RuntimeList() {
  const { items } = await j("/runtimes");
  page(`<h2>Cluster serving runtimes (${items.length})</h2><div class="row"><a class="btn" href="#runtimes/new">new runtime</a>
      <a class="btn sec" href="#runtimes/import">import</a></div><div id="t"></div>`);
  dataTable($("#t"), { name: "clusterservingruntimes", rows: items, href: (r) => `runtimes/${r.metadata.name}`, onDelete: (r) => del(`/runtimes/${enc(r.metadata.name)}`),
    cols: [["name", (r) => esc(r.metadata.name), (r) => r.metadata.name],
      ["formats", (r) => pills(fmtList(r)), (r) => fmtList(r).join(","), (r) => fmtList(r).join(" ")],
      ["size", (r) => esc(r.spec?.modelSizeRange ? `${r.spec.modelSizeRange.min || ""}–${r.spec.modelSizeRange.max || ""}` : ""), (r) => r.spec?.modelSizeRange?.min],
      ["protocols", (r) => pills(r.spec?.protocolVersions), (r) => (r.spec?.protocolVersions || []).join(",")],
      ["mode", (r) => esc(rtMode(r)), rtMode],
      ["GPUs", (r) => esc((r.spec?.engineConfig?.runner || r.spec?.engineConfig?.leader?.runner || {}).resources?.limits?.["amd.com/gpu"] ?? ""),
        (r) => Number((r.spec?.engineConfig?.runner || r.spec?.engineConfig?.leader?.runner || {}).resources?.limits?.["amd.com/gpu"] || 0)],
      ["state", (r) => (r.spec?.disabled ? badge("disabled") : badge("enabled")), (r) => (r.spec?.disabled ? 1 : 0)]] });
}
async function RuntimeDetail(name) {
  const r = await j(`/runtimes/${enc(name)}`);
  const sp = r.spec || {}, ec = sp.engineConfig || {};
  const runner = ec.runner || ec.leader?.runner || {};
  const cont = (c) => c ? kv([["image", `<code>${esc(c.image)}</code>`], ["command", `<code>${esc([...(c.command || []), ...(c.args || [])].join(" "))}</code>`],
    ["resources", esc(JSON.stringify(c.resources || {}))], ["env", esc((c.env || []).map((e) => `${e.name}=${e.value ?? ""}`).join("  "))]]) : `<p class="muted">none</p>`;
  page(`<h2>${esc(name)} ${sp.disabled ? badge("disabled") : badge("enabled")}</h2><div class="row"><a class="btn sec" href="#runtimes/${enc(name)}/edit">edit</a>
      <a class="btn sec" href="#runtimes/${enc(name)}/clone">clone</a><button class="btn sec" id="exp">export YAML</button><button class="btn" id="del">delete</button></div>
    ${kv([["mode", esc(rtMode(r))], ["model size range", esc(sp.modelSizeRange ? `${sp.modelSizeRange.min || ""} – ${sp.modelSizeRange.max || ""}` : "")],
      ["protocols", pills(sp.protocolVersions)], ["GPUs per pod", esc(runner.resources?.limits?.["amd.com/gpu"] ?? "")],
      ["workers", esc(ec.worker?.size ?? "")], ["accelerators", pills(sp.acceleratorRequirements?.acceleratorClasses)],
      ["cloned from", esc(r.metadata.annotations?.["ome.io/cloned-from"] || "")]])}
    <h3>Supported model formats</h3><div id="tf"></div>
    ${F.section("engine", cont(ec.runner || ec.leader?.runner))}${ec.worker ? F.section("worker", cont(ec.worker.runner), false) : ""}
    ${sp.decoderConfig ? F.section("decoder (PD)", cont(sp.decoderConfig.runner), false) : ""}${sp.routerConfig ? F.section("router", cont(sp.routerConfig.runner), false) : ""}
    <h3>Check a model against this runtime</h3><div class="row"><input id="mm" placeholder="model name"><button class="btn" id="chk">check</button></div><pre id="cres"></pre>
    <details class="sec"><summary>Object (YAML)</summary><pre>${esc(toYaml(r))}</pre></details>`);
  dataTable($("#tf"), { name: `${name}-formats`, rows: (sp.supportedModelFormats || []).map((f, i) => ({ ...f, metadata: { name: String(i) } })),
    cols: [["format", (f) => esc(`${f.modelFormat?.name || f.name || ""} ${f.modelFormat?.version || ""}`)],
      ["framework", (f) => esc(`${f.modelFramework?.name || ""} ${f.modelFramework?.version || ""}`)], ["architecture", (f) => esc(f.modelArchitecture || "")],
      ["quantization", (f) => esc(f.quantization || "")], ["autoSelect", (f) => esc(f.autoSelect ? "yes" : "no")], ["priority", (f) => esc(f.priority ?? ""), (f) => f.priority ?? -1]] });
  $("#exp").onclick = () => download(`${name}.yaml`, toYaml(cleanForEdit(r)) + "\n", "application/yaml");
  $("#chk").onclick = async () => { try { $("#cres").textContent = JSON.stringify(await j(`/runtimes/${enc(name)}/compatibility?model=${enc($("#mm").value)}`), null, 2); } catch (e) { showErr(e); } };
  $("#del").onclick = async () => { if (confirm(`delete ${name}?`)) { try { await del(`/runtimes/${enc(name)}`); location.hash = "runtimes"; } catch (e) { showErr(e); } } };
}
function RuntimeClone(name) {
  page(`<h2>Clone ${esc(name)}</h2><label>new name</label><input id="nn" size="40" value="${esc(name)}-copy">
    <p class="muted">The clone is created disabled (an identical enabled copy would tie its source's auto-select priority).</p>
    <button class="btn" id="go">clone</button>`);
  $("#go").onclick = async () => {
    const err = OME.validateName($("#nn").value);
    if (err) { showErr(new Error(err)); return; }
    try { await post(`/runtimes/${enc(name)}/clone`, { newName: $("#nn").value }); location.hash = `runtimes/${$("#nn").value}/edit`; } catch (e) { showErr(e); }
  };
}
function RuntimeNew() {
  let state = () => ({});
  const body = `<div id="rb" class="grid2">
      ${F.field("name", F.inp("name", "", "my-runtime", 32))}
      ${F.field("model size min / max", F.inp("sizeMin", "", "1B", 6) + " " + F.inp("sizeMax", "", "70B", 6))}
      ${F.chk("disabled", false, "disabled")} ${F.chk("multiNode", false, "multi-node (leader + workers)")}
      ${F.field("workers", F.inp("workers", "", "1", 4), "worker pods per group (multi-node)")}
      ${F.chk("pd", false, "prefill/decode disaggregation (decoder + router)")}</div>
    <label>protocols</label><div id="protos" class="row">${["openAI", "cohere", "openInference-v2", "grpc-v2"].map((p) => F.chk(`p:${p}`, p === "openAI", p)).join("")}</div>
    <label>accelerator classes</label><div id="accs" class="row"></div>
    ${F.section("supported model formats", `<div id="fmts"></div>`)}
    ${F.section("engine container", `<div id="eng"></div>`)}
    ${F.section("worker container (multi-node; defaults to the engine's)", `<div id="wrk"></div>`, false)}
    ${F.section("decoder container (PD)", `<div id="dec"></div>`, false)}
    ${F.section("router container (PD)", `<div id="rtr"></div>`, false)}
    ${F.section("volumes", `<div id="vols"></div>`, false)}${F.section("labels", `<div id="labels"></div>`, false)}`;
  const refresh = formPage({ title: "New cluster serving runtime", intro: `Structured form (reference runtimes/new) — or <a href="#runtimes/import">import</a> YAML.`,
    body, build: () => OME.buildRuntime(state()), errors: () => OME.runtimeErrors(state()),
    submit: async (obj) => { const r = await post("/runtimes", obj); location.hash = `runtimes/${r.metadata.name}`; } });
  const eng = F.ContainerForm($("#eng"), { image: "ome-amd:latest", command: ["python3", "-m", "ome_amd.runtime.server"], args: ["--model-path", "$(MODEL_PATH)"],
    resources: { limits: { "amd.com/gpu": "1" } } }, refresh);
  const wrk = F.ContainerForm($("#wrk"), {}, refresh), dec = F.ContainerForm($("#dec"), {}, refresh), rtr = F.ContainerForm($("#rtr"), {}, refresh);
  const fmts = F.FormatsEditor($("#fmts"), [{ formatName: "safetensors", formatVersion: "1.0.0", frameworkName: "transformers", autoSelect: true, priority: 1 }], refresh);
  const vols = F.VolumesEditor($("#vols"), [], refresh), labels = F.KVEditor($("#labels"), [], { addLabel: "label", onChange: refresh });
  j("/accelerators").then(({ items }) => { $("#accs").innerHTML = items.map((a) => F.chk(`a:${a.metadata.name}`, false, a.metadata.name)).join("") || `<span class="muted">none defined</span>`; }).catch(() => {});
  state = () => {
    const b = F.read($("#rb"));
    const on = (el, p) => Object.entries(F.read(el)).filter(([k, v]) => v && k.startsWith(p)).map(([k]) => k.slice(p.length));
    const w = wrk.value();
    return { ...b, protocols: on($("#protos"), "p:"), accelerators: on($("#accs"), "a:"), formats: fmts.value(), engine: eng.value(),
             worker: w.image ? w : undefined, decoder: b.pd ? dec.value() : undefined, router: b.pd ? rtr.value() : undefined,
             volumes: vols.value(), labels: labels.value() };
  };
  refresh();
}
async function RuntimeImport() {
  const cat = await j("/runtimes/catalog").catch(() => ({ files: [] }));
  page(`<h2>Import a serving runtime</h2><p class="muted">Pick a runtime from the catalog, give a GitHub URL of a runtime YAML (mapped onto the
      local catalog: the console runs without egress), or paste YAML.</p>
    <div class="row"><input id="url" size="70" placeholder="https://github.com/user/repo/blob/main/runtime.yaml"><button class="btn sec" id="fetch">fetch</button></div>
    <h3>Catalog (${(cat.files || []).length})</h3><div id="tc"></div>
    <h3>Or paste YAML directly</h3><textarea id="ed" placeholder="YAML content will appear here..."></textarea>
    <div class="row"><button class="btn sec" id="val">validate</button><button class="btn" id="go">import</button></div><pre id="out"></pre>`);
  const fetchPath = async (p) => {
    try { const r = await j(`/runtimes/fetch-yaml?path=${enc(OME.catalogPath(p))}`); $("#ed").value = r.yaml || toYaml(r.runtime); $("#ed").scrollIntoView(); } catch (e) { showErr(e); }
  };
  dataTable($("#tc"), { name: "runtime-catalog", rows: (cat.files || []).map((f) => ({ ...f, metadata: { name: f.path } })), rowId: (f) => f.path,
    cols: [["path", (f) => `<a href="javascript:void 0" data-p="${esc(f.path)}">${esc(f.path)}</a>`, (f) => f.path, (f) => f.path],
      ["runtime", (f) => esc(f.name || ""), (f) => f.name], ["installed", (f) => (f.installed ? badge("Ready") : ""), (f) => (f.installed ? 1 : 0)]] });
  $("#tc").addEventListener("click", (ev) => { const a = ev.target.closest("[data-p]"); if (a) fetchPath(a.dataset.p); });
  $("#fetch").onclick = () => fetchPath($("#url").value);
  $("#val").onclick = async () => { try { $("#out").textContent = JSON.stringify(await post("/validate/yaml", $("#ed").value, "application/yaml"), null, 2); } catch (e) { showErr(e); } };
  $("#go").onclick = async () => { try { const r = await post("/runtimes", $("#ed").value, "application/yaml"); location.hash = `runtimes/${r.metadata.name}`; } catch (e) { showErr(e); } };
}

// ---------------------------------------------------------------- services
const svcComps = (s) => Object.keys(s.status?.components || {});
async function ServiceList() {
  const { items } = await j(`/services${NS.query()}`);
  page(`<h2>Inference services (${items.length}${NS.get() === "all" ? "" : ` in ${esc(NS.get())}`})</h2><div class="row"><a class="btn" href="#services/deploy">deploy</a></div><div id="t"></div>`);
  dataTable($("#t"), { name: "inferenceservices", rows: items, href: (s) => `services/${s.metadata.namespace}/${s.metadata.name}`,
    onDelete: (s) => del(`/services/${enc(s.metadata.name)}?namespace=${enc(s.metadata.namespace)}`),
    cols: [["namespace", (s) => esc(s.metadata.namespace), (s) => s.metadata.namespace], ["name", (s) => esc(s.metadata.name), (s) => s.metadata.name],
      ["model", (s) => esc(s.spec?.model?.name), (s) => s.spec?.model?.name], ["runtime", (s) => esc(s.spec?.runtime?.name || s.status?.runtime || "(auto)")],
      ["components", (s) => pills(svcComps(s)), (s) => svcComps(s).join(","), (s) => svcComps(s).join(" ")],
      ["state", (s) => badge(ready(s)), ready, ready], ["url", (s) => esc(s.status?.url || "")],
      ["age", (s) => esc(ago(s.metadata.creationTimestamp)), (s) => -Date.parse(s.metadata.creationTimestamp || 0)]] });
}
async function ServiceDetail(ns, name) {
  const [s, st] = await Promise.all([j(`/services/${enc(name)}?namespace=${enc(ns)}`), j(`/services/${enc(name)}/status?namespace=${enc(ns)}`)]);
  const comps = Object.entries(s.status?.components || {}).map(([k, v]) => ({ ...v, metadata: { name: k } }));
  const ann = s.metadata.annotations || {};
  page(`<h2>${esc(ns)}/${esc(name)} ${badge(st.ready ? "Ready" : "NotReady")}</h2><div class="row">
      <a class="btn sec" href="#services/${enc(ns)}/${enc(name)}/edit">edit</a><a class="btn sec" href="#benchmarks/new?service=${enc(name)}&namespace=${enc(ns)}">benchmark</a>
      <button class="btn" id="del">delete</button></div>` +
    kv([["model", `<a href="#models/${enc(s.spec?.model?.name || "")}">${esc(s.spec?.model?.name)}</a>`],
      ["runtime", esc(s.spec?.runtime?.name || "(auto-selected)")], ["url", st.url ? `<code>${esc(st.url)}</code> ${copyBtn(st.url)}` : ""],
      ["deployment mode", esc(ann["ome.io/deploymentMode"] || "")], ["autoscaler", esc(ann["ome.io/autoscalerClass"] || "")],
      ["engine replicas", esc(`${s.spec?.engine?.minReplicas ?? ""} – ${s.spec?.engine?.maxReplicas ?? ""}`)]]) +
    `<h3>Components</h3><div id="tc"></div><h3>Conditions</h3><div id="tk"></div>
     <details class="sec"><summary>Object (YAML)</summary><pre>${esc(toYaml(s))}</pre></details>`);
  dataTable($("#tc"), { name: `${name}-components`, rows: comps,
    cols: [["component", (c) => esc(c.metadata.name)], ["ready", (c) => badge(c.ready || c.latestReadyRevision ? "Ready" : "-")], ["url", (c) => esc(c.url || "")]] });
  dataTable($("#tk"), { name: `${name}-conditions`, rows: (s.status?.conditions || []).map((c) => ({ ...c, metadata: { name: c.type } })),
    cols: [["type", (c) => esc(c.type)], ["status", (c) => badge(c.status)], ["reason", (c) => esc(c.reason || "")], ["message", (c) => esc(c.message || "")],
      ["since", (c) => esc(ago(c.lastTransitionTime))]] });
  wireCopy();
  $("#del").onclick = async () => { if (confirm(`delete ${ns}/${name}?`)) { try { await del(`/services/${enc(name)}?namespace=${enc(ns)}`); location.hash = "services"; } catch (e) { showErr(e); } } };
}
async function ServiceDeploy(query) {
  const models = (await j("/models")).items;
  const pre = query.get("model") || "", preNs = query.get("namespace") || (NS.get() === "all" ? "default" : NS.get());
  let state = () => ({});
  const body = `<div class="row"><span class="step on">1 model</span> → <span class="step" id="s2">2 runtime</span> → <span class="step" id="s3">3 scale</span></div>
    <div id="sb" class="grid2">
      ${F.field("model", F.sel("model", [["", "—"], ...models.map((m) => m.metadata.name)], pre))}
      ${F.field("runtime", `<span id="rtsel">${F.sel("runtime", [["", "(auto-select)"]], "")}</span>`)}
      ${F.field("namespace", F.sel("namespace", window.__namespaces || ["default"], preNs))}
      ${F.field("service name", F.inp("name", pre, "my-inference-service", 32))}
      ${F.field("engine replicas min / max", F.inp("min", "1", "1", 4) + " " + F.inp("max", "1", "1", 4))}
      ${F.field("GPUs per engine pod (override)", F.inp("gpus", "", "", 4))}
      ${F.field("deployment mode", F.sel("deploymentMode", [["", "(from runtime)"], "RawDeployment", "Serverless", "MultiNode", "PDDisaggregated", "MultiNodeRayVLLM"], ""))}
      ${F.chk("pd", false, "prefill/decode disaggregation (decoder + router)")}
      ${F.field("decoder replicas min / max", F.inp("dmin", "1", "1", 4) + " " + F.inp("dmax", "1", "1", 4))}</div>
    ${F.section("autoscaling", `<div id="ab" class="grid2">
      ${F.field("autoscaler class", F.sel("autoscaler", [["", "(default)"], "hpa", "keda", "external"], ""))}
      ${F.field("HPA metric", F.sel("metric", [["", "(default)"], "cpu", "memory"], ""))}
      ${F.field("target utilisation %", F.inp("target", "", "80", 4))}
      ${F.field("KEDA Prometheus server", F.inp("promServer", "", "http://prometheus:9090", 28))}
      ${F.field("KEDA query", F.inp("promQuery", "", "sum(rate(...))", 28))}
      ${F.field("KEDA threshold / operator", F.inp("threshold", "", "10", 5) + " " + F.sel("operator", [["", "(default)"], "GreaterThanOrEqual", "LessThanOrEqual"], ""))}</div>`, false)}
    ${F.section("engine environment", `<div id="env"></div>`, false)}`;
  const refresh = formPage({ title: "Deploy an inference service", body,
    build: () => OME.buildService(state()), errors: () => OME.serviceErrors(state()),
    submit: async (o) => { await post(`/services?namespace=${enc(o.metadata.namespace)}`, o); location.hash = `services/${o.metadata.namespace}/${o.metadata.name}`; } });
  const env = F.KVEditor($("#env"), [], { keyPh: "VAR_NAME", addLabel: "env var", onChange: refresh });
  state = () => ({ ...F.read($("#sb")), ...F.read($("#ab")), env: env.value() });
  const pickModel = async () => {
    const m = $('#sb [data-f="model"]').value;
    if (!m) return;
    const nm = $('#sb [data-f="name"]');
    if (!nm.value) nm.value = m;
    $("#s2").classList.add("on");
    const c = await j(`/runtimes/compatible?model=${enc(m)}`).catch(() => ({ runtimes: [] }));
    $("#rtsel").innerHTML = F.sel("runtime", [["", "(auto-select)"], ...(c.runtimes || []).map((r) => [r.runtime, `${r.runtime} — score ${r.score}`])], "");
    $("#s3").classList.add("on");
    refresh();
  };
  $('#sb [data-f="model"]').addEventListener("change", pickModel);
  if (pre) pickModel();
  refresh();
}

// ---------------------------------------------------------------- accelerators
async function AcceleratorList() {
  const { items } = await j("/accelerators");
  page(`<h2>Accelerator classes (${items.length})</h2><div id="t"></div>`);
  dataTable($("#t"), { name: "acceleratorclasses", rows: items, href: (a) => `accelerators/${a.metadata.name}`,
    cols: [["name", (a) => esc(a.metadata.name), (a) => a.metadata.name], ["vendor", (a) => esc(a.spec?.vendor), (a) => a.spec?.vendor],
      ["family / model", (a) => esc(`${a.spec?.family || ""} ${a.spec?.model || ""}`)],
      ["memory GB", (a) => esc(a.spec?.capabilities?.memoryGB), (a) => Number(a.spec?.capabilities?.memoryGB || 0)],
      ["compute", (a) => esc(a.spec?.capabilities?.computeCapability || "")],
      ["nodes", (a) => esc(a.status?.availableNodes?.length ?? a.status?.nodes?.length ?? ""), (a) => (a.status?.availableNodes || a.status?.nodes || []).length]] });
}
async function AcceleratorDetail(name) {
  const a = await j(`/accelerators/${enc(name)}`);
  const nodes = a.status?.availableNodes || a.status?.nodes || [];
  page(`<h2>${esc(name)}</h2>` + kv([["vendor", esc(a.spec?.vendor)], ["family", esc(a.spec?.family)], ["model", esc(a.spec?.model)]]) +
    `<h3>Capabilities</h3>` + kv(Object.entries(a.spec?.capabilities || {}).map(([k, v]) => [k, esc(typeof v === "object" ? JSON.stringify(v) : v)])) +
    `<h3>Nodes (${nodes.length})</h3>${pills(nodes.map((n) => (typeof n === "object" ? n.name || JSON.stringify(n) : n)))}
     <h3>Discovery</h3><pre>${esc(toYaml(a.spec?.discovery || {}))}</pre><details class="sec"><summary>Status</summary><pre>${esc(toYaml(a.status || {}))}</pre></details>`);
}

// ---------------------------------------------------------------- benchmarks
async function BenchmarkList() {
  const { items } = await j(`/benchmarks${NS.query()}`);
  const ep = (b) => b.spec?.endpoint?.inferenceService?.name || b.spec?.endpoint?.endpoint?.url || "";
  page(`<h2>Benchmark jobs (${items.length})</h2><div class="row"><a class="btn" href="#benchmarks/new">new benchmark</a></div><div id="t"></div>`);
  dataTable($("#t"), { name: "benchmarkjobs", rows: items, href: (b) => `benchmarks/${b.metadata.namespace}/${b.metadata.name}`,
    onDelete: (b) => del(`/benchmarks/${enc(b.metadata.name)}?namespace=${enc(b.metadata.namespace)}`),
    cols: [["namespace/name", (b) => esc(`${b.metadata.namespace}/${b.metadata.name}`), (b) => b.metadata.name], ["endpoint", (b) => esc(ep(b)), ep],
      ["task", (b) => esc(b.spec?.task), (b) => b.spec?.task], ["scenarios", (b) => pills(b.spec?.trafficScenarios), (b) => (b.spec?.trafficScenarios || []).join(",")],
      ["concurrency", (b) => esc((b.spec?.numConcurrency || []).join(","))], ["state", (b) => badge(b.status?.state || ready(b)), (b) => b.status?.state || ready(b)],
      ["age", (b) => esc(ago(b.metadata.creationTimestamp)), (b) => -Date.parse(b.metadata.creationTimestamp || 0)]] });
}
async function BenchmarkNew(query) {
  const svcs = (await j(`/services${NS.query()}`)).items;
  const preSvc = query.get("service") || "", preNs = query.get("namespace") || (NS.get() === "all" ? "default" : NS.get());
  let state = () => ({});
  const body = `<div id="bb" class="grid2">
      ${F.field("name", F.inp("name", preSvc ? `${preSvc}-bench` : "", "bench", 28))}
      ${F.field("namespace", F.sel("namespace", window.__namespaces || ["default"], preNs))}
      ${F.field("inference service", F.sel("service", [["", "—"], ...svcs.map((s) => [s.metadata.name, `${s.metadata.namespace}/${s.metadata.name}`])], preSvc))}
      ${F.field("or endpoint URL", F.inp("url", "", "http://host:8080", 28))}
      ${F.field("API format / model name", F.sel("apiFormat", ["openai", "cohere"], "openai") + " " + F.inp("modelName", "", "", 16))}
      ${F.field("task", F.sel("task", ["text-to-text", "text-to-embeddings", "image-text-to-text", "text-to-rerank"], "text-to-text"))}
      ${F.field("traffic scenarios", F.inp("scenarios", "N(480,240)/(300,150) D(100,100)", "", 36), "space-separated; N(μin,σin)/(μout,σout), D(in,out), U(...), E(tokens)")}
      ${F.field("concurrency", F.inp("concurrency", "1 8 64 256", "", 20))}
      ${F.field("max time / requests per iteration", F.inp("maxTime", "15", "", 5) + " " + F.inp("maxRequests", "100", "", 5))}
      ${F.field("results location", F.inp("output", "local:///tmp/ome-bench-results", "", 36))}</div>`;
  const refresh = formPage({ title: "New benchmark job", body, build: () => OME.buildBenchmark(state()),
    errors: () => { const s = state(), e = []; const n = OME.validateName(s.name); if (n) e.push(n); if (!s.service && !s.url) e.push("an inference service or an endpoint URL is required"); return e; },
    submit: async (o) => { await post(`/benchmarks?namespace=${enc(o.metadata.namespace)}`, o); location.hash = `benchmarks/${o.metadata.namespace}/${o.metadata.name}`; } });
  state = () => { const b = F.read($("#bb")); return { ...b, serviceNamespace: (svcs.find((s) => s.metadata.name === b.service) || { metadata: {} }).metadata.namespace }; };
  refresh();
}
async function BenchmarkDetail(ns, name) {
  const b = await j(`/benchmarks/${enc(name)}?namespace=${enc(ns)}`);
  const res = b.status?.results || b.status?.summary;
  page(`<h2>${esc(ns)}/${esc(name)} ${badge(b.status?.state || ready(b))}</h2><div class="row"><button class="btn" id="del">delete</button></div>` +
    kv([["task", esc(b.spec?.task)], ["scenarios", pills(b.spec?.trafficScenarios)], ["concurrency", esc((b.spec?.numConcurrency || []).join(", "))],
      ["results", esc(b.spec?.outputLocation?.storageUri || "")], ["started", esc(b.status?.startTime || "")], ["finished", esc(b.status?.completionTime || "")],
      ["details", esc(b.status?.details || "")]]) +
    (res ? `<h3>Results</h3><pre>${esc(typeof res === "string" ? res : toYaml(res))}</pre>` : "") +
    `<details class="sec" open><summary>Status</summary><pre>${esc(toYaml(b.status || {}))}</pre></details>`);
  $("#del").onclick = async () => { if (confirm(`delete ${ns}/${name}?`)) { try { await del(`/benchmarks/${enc(name)}?namespace=${enc(ns)}`); location.hash = "benchmarks"; } catch (e) { showErr(e); } } };
}
function Validate() {
  page(`<h2>Validate manifests</h2><p class="muted">Runs the manager's admission chain (defaulting + validation) without persisting.</p>
    <textarea id="ed">apiVersion: ome.io/v1beta1\nkind: InferenceService\nmetadata:\n  name: llama3-8b\n  namespace: default\nspec:\n  model:\n    name: llama-3-8b-instruct\n</textarea>
    <div class="row"><button class="btn" id="val">validate</button></div><pre id="out"></pre>`);
  $("#val").onclick = async () => { try { $("#out").textContent = JSON.stringify(await post("/validate/yaml", $("#ed").value, "application/yaml"), null, 2); } catch (e) { showErr(e); } };
}

// ---------------------------------------------------------------- router
const ROUTES = [
  [/^$|^dashboard$/, Dashboard, "dashboard"],
  [/^models$/, ModelList, "models"], [/^models\/new$/, ModelNew, "models"], [/^models\/import$/, ModelImport, "models"],
  [/^models\/ns\/([^/]+)\/([^/]+)\/edit$/, editor((ns, n) => `/namespaces/${enc(ns)}/models/${enc(n)}`, (ns, n) => `models/ns/${ns}/${n}`), "models"],
  [/^models\/ns\/([^/]+)\/([^/]+)$/, ModelDetail, "models"],
  [/^models\/([^/]+)\/edit$/, editor((n) => `/models/${enc(n)}`, (n) => `models/${n}`), "models"], [/^models\/([^/]+)$/, ModelDetail, "models"],
  [/^runtimes$/, RuntimeList, "runtimes"], [/^runtimes\/new$/, RuntimeNew, "runtimes"], [/^runtimes\/import$/, RuntimeImport, "runtimes"],
  [/^runtimes\/([^/]+)\/clone$/, RuntimeClone, "runtimes"], [/^runtimes\/([^/]+)\/edit$/, editor((n) => `/runtimes/${enc(n)}`, (n) => `runtimes/${n}`), "runtimes"],
  [/^runtimes\/([^/]+)$/, RuntimeDetail, "runtimes"],
  [/^services$/, ServiceList, "services"], [/^services\/deploy$/, ServiceDeploy, "services", true],
  [/^services\/([^/]+)\/([^/]+)\/edit$/, editor((ns, n) => `/services/${enc(n)}?namespace=${enc(ns)}`, (ns, n) => `services/${ns}/${n}`), "services"],
  [/^services\/([^/]+)\/([^/]+)$/, ServiceDetail, "services"],
  [/^accelerators$/, AcceleratorList, "accelerators"], [/^accelerators\/([^/]+)$/, AcceleratorDetail, "accelerators"],
  [/^benchmarks$/, BenchmarkList, "benchmarks"], [/^benchmarks\/new$/, BenchmarkNew, "benchmarks", true],
  [/^benchmarks\/([^/]+)\/([^/]+)$/, BenchmarkDetail, "benchmarks"],
  [/^validate$/, Validate, "validate"],
];
const NAV = ["dashboard", "models", "runtimes", "services", "accelerators", "benchmarks", "validate"];
function route() {
  const [path, qs] = location.hash.slice(1).split("?");
  const query = new URLSearchParams(qs || "");
  for (const [re, fn, tab, wantsQuery] of ROUTES) {
    const m = path.match(re);
    if (!m) continue;
    $("#nav").innerHTML = NAV.map((t) => `<a href="#${t}" class="${t === tab ? "on" : ""}">${t}</a>`).join("");
    const args = m.slice(1).filter((x) => x !== undefined).map(decodeURIComponent);
    Promise.resolve(wantsQuery ? fn(query) : fn(...args)).catch((e) => page(`<div class="err">${esc(e.message)}</div>`));
    return;
  }
  location.hash = "dashboard";
}
window.onhashchange = route;
fetch("health").then((r) => r.json()).then((h) => { $("#health").textContent = `api ${h.status}`; }).catch(() => { $("#health").textContent = "api unreachable"; });
const es = new EventSource(`${API}/events`);
es.addEventListener("connected", () => { $("#conn").textContent = "connected"; });
es.onerror = () => { $("#conn").textContent = "reconnecting…"; };
let pending = null;
for (const t of ["add", "update", "delete"]) es.addEventListener(t, (ev) => {
  const m = JSON.parse(ev.data);
  $("#feed").insertAdjacentHTML("afterbegin", `<div><span class="${t === "delete" ? "bad" : t === "add" ? "ok" : "muted"}">${t}</span> ${esc(m.resource)} ${esc(m.namespace ? m.namespace + "/" : "")}${esc(m.name)}</div>`);
  const cur = location.hash.slice(1).split("/")[0] || "dashboard";
  const busy = ["/edit", "/new", "deploy", "/import", "/clone"].some((s) => location.hash.includes(s));
  if ((cur === m.resource || cur === "dashboard") && !busy) { clearTimeout(pending); pending = setTimeout(route, 300); }   // coalesce bursts
});
loadNamespaces().then((ns) => { window.__namespaces = ns; route(); });
