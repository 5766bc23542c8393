// ome-amd web console — form widgets for the structured create / edit views (reference
// web-console/frontend/src/components/forms: FormField / FormInput / FormSelect, ContainerForm,
// VolumeForm, storage/*, runtime/*, CollapsibleSection).  Each widget renders into a container
// element and exposes value(); manifests are assembled by lib.js (OME.build*).
"use strict";
(function (root) {
  const { esc, SCHEMES, buildUri, parseUri } = root.OME;
  const q = (s, el) => el.querySelector(s);
  const qa = (s, el) => [...el.querySelectorAll(s)];
  let uid = 0;
  const nid = (p) => `${p}${++uid}`;

  function inp(name, value, ph = "", size = 24, type = "text") {
    return `<input data-f="${esc(name)}" type="${type}" size="${size}" value="${esc(value == null ? "" : value)}" placeholder="${esc(ph)}">`;
  }
  function sel(name, options, value) {
    return `<select data-f="${esc(name)}">${options.map((o) => {
      const [v, l] = Array.isArray(o) ? o : [o, o];
      return `<option value="${esc(v)}" ${String(v) === String(value == null ? "" : value) ? "selected" : ""}>${esc(l)}</option>`;
    }).join("")}</select>`;
  }
  function chk(name, on, label) { return `<label class="inl"><input type="checkbox" data-f="${esc(name)}" ${on ? "checked" : ""}> ${esc(label)}</label>`; }
  function field(label, html, help) { return `<div class="fld"><label>${esc(label)}</label>${html}${help ? `<div class="help">${esc(help)}</div>` : ""}</div>`; }
  function section(title, body, open = true) { return `<details class="sec" ${open ? "open" : ""}><summary>${esc(title)}</summary><div class="secb">${body}</div></details>`; }
  function read(el) {   // {data-f name: value} of every field directly inside el
    const o = {};
    qa("[data-f]", el).forEach((x) => { o[x.dataset.f] = x.type === "checkbox" ? x.checked : x.value; });
    return o;
  }

  // key/value list (env vars, labels, node selectors, parameters)
  function KVEditor(el, pairs = [], opt = {}) {
    const kph = opt.keyPh || "Key", vph = opt.valPh || "Value";
    const row = (k = "", v = "") => `<div class="kvrow">${inp("k", k, kph, 20)} ${inp("v", v, vph, 28)} <button class="btn sec x" type="button">×</button></div>`;
    el.innerHTML = `<div class="kvrows">${pairs.map(([k, v]) => row(k, v)).join("")}</div><button class="btn sec" type="button" data-add>+ ${esc(opt.addLabel || "add")}</button>`;
    const rows = q(".kvrows", el);
    const wireX = () => qa(".x", rows).forEach((b) => { b.onclick = () => { b.parentElement.remove(); if (opt.onChange) opt.onChange(); }; });
    q("[data-add]", el).onclick = () => { rows.insertAdjacentHTML("beforeend", row()); wireX(); };
    el.oninput = () => { if (opt.onChange) opt.onChange(); };
    wireX();
    return { value: () => qa(".kvrow", rows).map((r) => [q('[data-f="k"]', r).value, q('[data-f="v"]', r).value]).filter(([k]) => k.trim()) };
  }

  // storage URI builder: scheme + that scheme's fields, or a raw URI
  function StorageBuilder(el, uri = "", onChange) {
    const p = parseUri(uri);
    let scheme = p ? p.scheme : "hf";
    const fieldsHtml = (s, vals = {}) => SCHEMES[s].fields.map(([k, ph]) => field(k, inp(k, vals[k] || "", ph, 36))).join("");
    el.innerHTML = `<div class="row">${sel("scheme", Object.entries(SCHEMES).map(([k, v]) => [k, `${k}:// — ${v.label}`]), scheme)}
      ${chk("raw", false, "edit the URI directly")}</div><div class="sfields">${fieldsHtml(scheme, p ? p.fields : {})}</div>
      <div class="rawbox" hidden>${inp("uri", uri, "hf://org/model", 60)}</div><div class="help">URI: <code class="uri"></code></div>`;
    const sf = q(".sfields", el), rawbox = q(".rawbox", el), raw = q('[data-f="raw"]', el);
    const value = () => {
      if (raw.checked) return q('[data-f="uri"]', rawbox).value.trim();
      try { return buildUri(scheme, read(sf)); } catch (e) { return ""; }
    };
    const upd = () => { q(".uri", el).textContent = value(); if (onChange) onChange(); };
    q('[data-f="scheme"]', el).onchange = (ev) => { scheme = ev.target.value; sf.innerHTML = fieldsHtml(scheme); upd(); };
    raw.onchange = () => {
      if (raw.checked) q('[data-f="uri"]', rawbox).value = buildUri(scheme, read(sf));
      else { const pp = parseUri(q('[data-f="uri"]', rawbox).value); if (pp) { scheme = pp.scheme; q('[data-f="scheme"]', el).value = scheme; sf.innerHTML = fieldsHtml(scheme, pp.fields); } }
      rawbox.hidden = !raw.checked; sf.hidden = raw.checked; upd();
    };
    sf.oninput = upd; rawbox.oninput = upd;
    upd();
    return { value };
  }

  // container (runner) form: image, command/args, env, resources, port
  function ContainerForm(el, c = {}, onChange) {
    const lim = (c.resources && c.resources.limits) || {}, req = (c.resources && c.resources.requests) || {};
    const envId = nid("env");
    el.innerHTML = `<div class="grid2">
        ${field("container name", inp("name", c.name || "ome-container", "container-name"))}
        ${field("image", inp("image", c.image || "", "image:tag", 40))}
        ${field("command", inp("command", (c.command || []).join(" "), "/bin/sh", 40), "space-separated")}
        ${field("args", inp("args", (c.args || []).join(" "), "--arg=value", 40), "space-separated")}
        ${field("GPUs (amd.com/gpu)", inp("gpus", lim["amd.com/gpu"] || "", "1", 6))}
        ${field("port", inp("port", (c.ports && c.ports[0] && c.ports[0].containerPort) || "", "8080", 6))}
        ${field("CPU request / limit", inp("cpu", req.cpu || "", "1000m", 8) + " " + inp("cpuLimit", lim.cpu || "", "", 8))}
        ${field("memory request / limit", inp("memory", req.memory || "", "128Mi", 8) + " " + inp("memoryLimit", lim.memory || "", "512Mi", 8))}
      </div><label>environment</label><div id="${envId}"></div>`;
    const env = KVEditor(q(`#${envId}`, el), (c.env || []).map((e) => [e.name, e.value]), { keyPh: "VAR_NAME", valPh: "value", addLabel: "env var", onChange });
    el.oninput = () => { if (onChange) onChange(); };
    return { value: () => ({ ...read(q(".grid2", el)), env: env.value() }) };
  }

  // supported model formats of a runtime
  const QUANT = ["", "fp8", "fbgemm_fp8", "int8", "int4", "mxfp4", "gptq", "awq"];
  function FormatsEditor(el, rows = [], onChange) {
    const row = (x = {}) => `<tr>
      <td>${inp("formatName", x.formatName || (x.modelFormat && x.modelFormat.name) || "", "safetensors", 11)}</td>
      <td>${inp("formatVersion", x.formatVersion || (x.modelFormat && x.modelFormat.version) || "", "1.0.0", 6)}</td>
      <td>${inp("frameworkName", x.frameworkName || (x.modelFramework && x.modelFramework.name) || "", "transformers", 11)}</td>
      <td>${inp("frameworkVersion", x.frameworkVersion || (x.modelFramework && x.modelFramework.version) || "", "4.46.0", 6)}</td>
      <td>${inp("architecture", x.architecture || x.modelArchitecture || "", "LlamaForCausalLM", 18)}</td>
      <td>${sel("quantization", QUANT, x.quantization || "")}</td>
      <td><input type="checkbox" data-f="autoSelect" ${x.autoSelect ? "checked" : ""}></td>
      <td>${inp("priority", x.priority == null ? "" : x.priority, "1", 3)}</td>
      <td><button class="btn sec x" type="button">×</button></td></tr>`;
    el.innerHTML = `<table class="ftab"><tr><th>format</th><th>version</th><th>framework</th><th>version</th><th>architecture</th>
      <th>quant</th><th>auto</th><th>prio</th><th></th></tr>${(rows.length ? rows : [{}]).map(row).join("")}</table>
      <button class="btn sec" type="button" data-add>+ format</button>`;
    const tab = q("table", el);
    const wireX = () => qa(".x", tab).forEach((b) => { b.onclick = () => { b.closest("tr").remove(); if (onChange) onChange(); }; });
    q("[data-add]", el).onclick = () => { tab.insertAdjacentHTML("beforeend", row()); wireX(); };
    el.oninput = () => { if (onChange) onChange(); };
    el.onchange = el.oninput;
    wireX();
    return { value: () => qa("tr", tab).slice(1).map(read) };
  }

  // volumes: emptyDir / hostPath / PVC
  function VolumesEditor(el, vols = [], onChange) {
    const row = (v = {}) => `<div class="kvrow">${inp("name", v.name || "", "volume-name", 14)}
      ${inp("claim", (v.persistentVolumeClaim && v.persistentVolumeClaim.claimName) || "", "pvc claim (or)", 14)}
      ${inp("hostPath", (v.hostPath && v.hostPath.path) || "", "/mnt/path (or)", 14)}
      ${sel("medium", [["", "emptyDir"], ["Memory", "emptyDir (Memory)"]], (v.emptyDir && v.emptyDir.medium) || "")}
      <button class="btn sec x" type="button">×</button></div>`;
    el.innerHTML = `<div class="kvrows">${vols.map(row).join("")}</div><button class="btn sec" type="button" data-add>+ volume</button>`;
    const rows = q(".kvrows", el);
    const wireX = () => qa(".x", rows).forEach((b) => { b.onclick = () => { b.parentElement.remove(); if (onChange) onChange(); }; });
    q("[data-add]", el).onclick = () => { rows.insertAdjacentHTML("beforeend", row()); wireX(); };
    el.oninput = () => { if (onChange) onChange(); };
    wireX();
    return { value: () => qa(".kvrow", rows).map(read) };
  }

  root.OMEForms = { inp, sel, chk, field, section, read, KVEditor, StorageBuilder, ContainerForm, FormatsEditor, VolumesEditor, QUANT };
})(typeof globalThis !== "undefined" ? globalThis : this);
