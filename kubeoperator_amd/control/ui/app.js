// KubeOperator-AMD web UI: a dependency-free single-page app over /api/v1 and the two websockets.
// Module map follows the reference UI (SURVEY.md §2.9): sign-in, dashboard, clusters (list, create wizard
// with device checks, detail tabs: overview / nodes / deploy progress + live log / health / events / backup /
// grade / configs), hosts (+import), credentials, regions / zones / plans, packages, NFS / Ceph, items + members
// + resources, users, settings (system, backup storage, LDAP, notification), message center, system log.
"use strict";

const API = "/api/v1";
const $ = (sel, el = document) => el.querySelector(sel);
const esc = (s) => String(s ?? "").replace(/[&<>"']/g, (c) => ({"&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;"}[c]));
const st = (s) => `<span class="status ${esc(s)}">${esc(s)}</span>`;
let ME = null;

// ------------------------------------------------------------------ API client (JWT header, refresh)
async function api(method, path, body, opts = {}) {
  const headers = {};
  const tok = localStorage.getItem("kop_token");
  if (tok) headers.Authorization = "JWT " + tok;
  let payload;
  if (body instanceof FormData) payload = body;
  else if (body !== undefined) { headers["Content-Type"] = "application/json"; payload = JSON.stringify(body); }
  const r = await fetch(API + path, {method, headers, body: payload});
  if (r.status === 401 && !opts.noAuthRedirect) { logout(); throw new Error("session expired"); }
  if (opts.raw) return r;
  const text = await r.text();
  const data = text ? (() => { try { return JSON.parse(text); } catch { return text; } })() : null;
  if (!r.ok) throw new Error((data && (data.detail || JSON.stringify(data))) || r.statusText);
  return data;
}
const GET = (p) => api("GET", p), POST = (p, b) => api("POST", p, b ?? {}), PUT = (p, b) => api("PUT", p, b ?? {}),
  PATCH = (p, b) => api("PATCH", p, b ?? {}), DEL = (p) => api("DELETE", p);

function wsURL(path) { return (location.protocol === "https:" ? "wss://" : "ws://") + location.host + path; }

async function refreshToken() {
  const tok = localStorage.getItem("kop_token");
  if (!tok) return;
  try { const r = await api("POST", "/token/refresh/", {token: tok}, {noAuthRedirect: true}); localStorage.setItem("kop_token", r.token); }
  catch { /* expired: next call redirects */ }
}

// ------------------------------------------------------------------ auth
function logout() { localStorage.removeItem("kop_token"); ME = null; showLogin(); }
function showLogin() { $("#shell").classList.add("hidden"); $("#login").classList.remove("hidden"); }
$("#login-form").addEventListener("submit", async (e) => {
  e.preventDefault();
  const f = new FormData(e.target);
  try {
    const r = await api("POST", "/token/auth/", {username: f.get("username"), password: f.get("password")}, {noAuthRedirect: true});
    localStorage.setItem("kop_token", r.token);
    $("#login-error").textContent = "";
    boot();
  } catch (err) { $("#login-error").textContent = err.message; }
});
$("#logout").onclick = logout;

// ------------------------------------------------------------------ helpers: tables, forms, modal
function table(rows, cols, empty = "Nothing here yet.") {
  if (!rows || !rows.length) return `<p class="muted">${empty}</p>`;
  return `<table><tr>${cols.map((c) => `<th>${esc(c[0])}</th>`).join("")}</tr>${rows.map((r) =>
    `<tr>${cols.map((c) => `<td>${typeof c[1] === "function" ? c[1](r) : esc(r[c[1]])}</td>`).join("")}</tr>`).join("")}</table>`;
}
function kv(obj) {
  return `<table class="kv">${Object.entries(obj).map(([k, v]) => `<tr><td>${esc(k)}</td><td>${typeof v === "object" ? `<code>${esc(JSON.stringify(v))}</code>` : esc(v)}</td></tr>`).join("")}</table>`;
}
function modal(html) { $("#modal-body").innerHTML = html; $("#modal").classList.remove("hidden"); }
function closeModal() { $("#modal").classList.add("hidden"); }
$("#modal").addEventListener("click", (e) => { if (e.target.id === "modal") closeModal(); });

// fields: [name, label, type("text"|"password"|"number"|"select"|"textarea"|"json"|"checkbox"), options|default]
function formModal(title, fields, onSubmit, initial = {}) {
  const inputs = fields.map(([name, label, type = "text", opt]) => {
    const v = initial[name] ?? (type === "select" ? "" : (opt ?? ""));
    if (type === "select") return `<label>${esc(label)}<select name="${name}">${(opt || []).map((o) => {
      const [val, txt] = Array.isArray(o) ? o : [o, o];
      return `<option value="${esc(val)}" ${String(val) === String(v) ? "selected" : ""}>${esc(txt)}</option>`; }).join("")}</select></label>`;
    if (type === "textarea" || type === "json") return `<label>${esc(label)}<textarea name="${name}">${esc(type === "json" ? JSON.stringify(v || {}, null, 2) : v)}</textarea></label>`;
    if (type === "checkbox") return `<label><input type="checkbox" name="${name}" style="width:auto" ${v ? "checked" : ""}> ${esc(label)}</label>`;
    return `<label>${esc(label)}<input name="${name}" type="${type}" value="${esc(v)}"></label>`;
  }).join("");
  modal(`<h2>${esc(title)}</h2><form id="mf">${inputs}<div class="toolbar"><button type="submit">OK</button>
    <button type="button" class="secondary" onclick="closeModal()">Cancel</button></div><p class="error" id="mf-err"></p></form>`);
  $("#mf").addEventListener("submit", async (e) => {
    e.preventDefault();
    const out = {};
    for (const [name, , type] of fields) {
      const el = e.target.elements[name];
      if (type === "number") out[name] = el.value === "" ? null : Number(el.value);
      else if (type === "json") { try { out[name] = JSON.parse(el.value || "{}"); } catch (err) { $("#mf-err").textContent = `${name}: ${err.message}`; return; } }
      else if (type === "checkbox") out[name] = el.checked;
      else out[name] = el.value;
    }
    // a submit that navigates (an operation opening its deploy tab) is rendered by the hashchange alone: a second
    // route() here would render the same view twice, concurrently
    try { const h = location.hash; await onSubmit(out); closeModal(); if (location.hash === h) route(); } catch (err) { $("#mf-err").textContent = err.message; }
  });
}
async function confirmDo(text, fn) { if (confirm(text)) { try { await fn(); route(); } catch (e) { alert(e.message); } } }

// generic CRUD page for simple resources
function crudPage(title, path, cols, fields, opts = {}) {
  return async (v) => {
    const rows = await GET(path);
    const list = Array.isArray(rows) ? rows : rows.results;
    v.innerHTML = `<h2>${esc(title)}</h2><div class="toolbar">${opts.readonly ? "" : `<button id="add">Add</button>`}${opts.extraButtons || ""}</div>
      ${table(list, [...cols, ...(opts.readonly ? [] : [["", (r) => `<button class="link" data-edit="${esc(r.id)}">edit</button><button class="link" data-del="${esc(r.id)}">delete</button>`]])])}`;
    if (opts.readonly) return;
    $("#add").onclick = () => formModal(`Add ${title}`, fields, (d) => POST(path, opts.prepare ? opts.prepare(d) : d));
    v.querySelectorAll("[data-edit]").forEach((b) => b.onclick = () => {
      const row = list.find((r) => r.id === b.dataset.edit);
      formModal(`Edit ${title}`, fields, (d) => PATCH(`${path}${row.id}/`, opts.prepare ? opts.prepare(d) : d), row);
    });
    v.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo("Delete?", () => DEL(`${path}${b.dataset.del}/`)));
    if (opts.after) opts.after(v, list);
  };
}

// ------------------------------------------------------------------ views
const views = {};

// dashboard (reference dashboard.component.html): item / cluster filters, cluster status, capacity (CPU, memory,
// AMD GPUs), statistics (nodes, pods, namespaces, deployments), warnings, restarting and failing pods. The monitor
// collects every 5 minutes (domain/monitor.py); "refresh" re-reads it.
views.dashboard = async (v, [item = "all", cluster = "all"]) => {
  const [clusters, hosts, items] = await Promise.all([GET("/clusters/"), GET("/host/"), GET("/items/").catch(() => [])]);
  const dash = await GET(`/dashboard/${encodeURIComponent(cluster)}/${encodeURIComponent(item)}/`).catch(() => ({clusters: []}));
  const gpus = hosts.reduce((a, h) => a + (h.gpu_num || 0), 0);
  const running = clusters.filter((c) => c.status === "RUNNING").length;
  const data = dash.clusters || [];
  const sum = (k) => data.reduce((a, d) => a + ((d[k] || []).length || 0), 0);
  const pct = (x) => `${Math.round(100 * (x || 0))} %`;
  const shown = item === "all" ? clusters : clusters.filter((c) => c.item_name === item);
  v.innerHTML = `<h2>Dashboard</h2><div class="toolbar"><select id="d-item" style="width:auto"><option value="all">all items</option>
      ${items.map((i) => `<option ${i.name === item ? "selected" : ""}>${esc(i.name)}</option>`).join("")}</select>
    <select id="d-cluster" style="width:auto"><option value="all">all clusters</option>${shown.map((c) => `<option ${c.name === cluster ? "selected" : ""}>${esc(c.name)}</option>`).join("")}</select>
    <button id="d-refresh" class="secondary">refresh</button><span class="muted">monitoring data every 5 minutes</span></div>
    <div class="grid">
    <div class="card stat"><div class="v">${clusters.length}</div><div class="k">clusters (${running} running)</div></div>
    <div class="card stat"><div class="v">${hosts.length}</div><div class="k">hosts</div></div>
    <div class="card stat"><div class="v">${gpus}</div><div class="k">AMD Instinct GPUs registered</div></div>
    <div class="card stat"><div class="v">${dash.gpu_allocatable ?? 0}/${dash.gpu_total ?? 0}</div><div class="k">amd.com/gpu allocatable / capacity</div></div>
    </div><h3>Cluster status</h3>${table(shown, [["Name", (c) => `<a href="#/cluster/${esc(c.name)}">${esc(c.name)}</a>`], ["Status", (c) => st(c.status)],
      ["Template", "template"], ["Nodes", "node_size"], ["GPUs", "gpu_num"], ["Package", "package"]])}
    <h3>Capacity</h3>${table(data, [["Cluster", "name"], ["CPU used", (d) => pct(d.cpu_usage)], ["Memory used", (d) => pct(d.mem_usage)],
      ["amd.com/gpu", (d) => `${esc(d.gpu_allocatable ?? 0)} / ${esc(d.gpu_total ?? 0)}`], ["Collected", "date"]], "No monitoring data yet.")}
    <h3>Statistics</h3><div class="grid">
      <div class="card stat"><div class="v">${sum("nodes")}</div><div class="k">nodes</div></div>
      <div class="card stat"><div class="v">${sum("pods")}</div><div class="k">pods</div></div>
      <div class="card stat"><div class="v">${sum("namespaces")}</div><div class="k">namespaces</div></div>
      <div class="card stat"><div class="v">${sum("deployments")}</div><div class="k">deployments</div></div></div>
    <h3>Warnings</h3>${table(dash.warn_containers || [], [["Cluster / node", (w) => esc(w.cluster || w.node || w.name || "")], ["Check", (w) => esc(w.type || w.reason || "")],
      ["Detail", (w) => esc(w.message || JSON.stringify(w))]], "No warnings.")}
    <h3>Pods restarting</h3>${table(dash.restart_pods || [], [["Namespace", "namespace"], ["Pod", "name"], ["Status", "status"], ["Restarts", "restart_count"]], "None.")}
    <h3>Pods failing</h3>${table(dash.error_pods || [], [["Namespace", "namespace"], ["Pod", "name"], ["Status", "status"], ["Restarts", "restart_count"]], "All pods healthy (or no monitoring data yet).")}`;
  $("#d-item").onchange = (e) => { location.hash = `#/dashboard/${encodeURIComponent(e.target.value)}/all`; };
  $("#d-cluster").onchange = (e) => { location.hash = `#/dashboard/${encodeURIComponent(item)}/${encodeURIComponent(e.target.value)}`; };
  $("#d-refresh").onclick = async () => {
    for (const c of cluster === "all" ? shown : shown.filter((x) => x.name === cluster)) await POST(`/cluster/${c.name}/monitor/refresh/`).catch(() => null);
    route();
  };
};

views.clusters = async (v) => {
  const rows = await GET("/clusters/");
  v.innerHTML = `<h2>Clusters</h2><div class="toolbar"><button id="new">Create cluster</button></div>
    ${table(rows, [["Name", (c) => `<a href="#/cluster/${esc(c.name)}">${esc(c.name)}</a>`], ["Status", (c) => st(c.status)], ["Template", "template"],
      ["Deploy", "deploy_type"], ["Nodes", "node_size"], ["GPUs", "gpu_num"], ["Package", "package"], ["Item", "item_name"],
      ["", (c) => `<button class="link" data-del="${esc(c.name)}">delete</button>`]])}`;
  $("#new").onclick = () => { location.hash = "#/cluster-create"; };
  v.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo(`Delete cluster ${b.dataset.del}?`, () => DEL(`/clusters/${b.dataset.del}/`)));
};

// create wizard: template -> package -> network -> storage -> nodes -> device checks (cluster-create.component.ts)
views["cluster-create"] = async (v) => {
  const [plan, pkgs, hosts, items, plans] = await Promise.all([GET("/cluster/config"), GET("/packages/"), GET("/host/"), GET("/items/"), GET("/plans/")]);
  const free = hosts.filter((h) => !h.node_id);
  const tmpls = plan.templates || [];
  v.innerHTML = `<h2>Create cluster</h2><form id="cc" class="card">
    <div class="row"><label>Name<input name="name" required pattern="[a-zA-Z0-9-]+"></label>
      <label>Item<select name="item_name">${items.map((i) => `<option>${esc(i.name)}</option>`).join("")}</select></label></div>
    <div class="row"><label>Template<select name="template">${tmpls.map((t) => `<option value="${esc(t.name)}">${esc(t.name)}${t.comment ? " — " + esc(t.comment) : ""}</option>`).join("")}</select></label>
      <label>Package<select name="package">${pkgs.map((p) => `<option value="${esc(p.name)}">${esc(p.name)} (${esc(p.meta.version || "")})</option>`).join("")}</select></label></div>
    <div class="row"><label>Deploy type<select name="deploy_type"><option>MANUAL</option><option>AUTOMATIC</option></select></label>
      <label>IaaS plan (AUTOMATIC)<select name="plan"><option value="">—</option>${plans.map((p) => `<option value="${esc(p.id)}">${esc(p.name)}</option>`).join("")}</select></label>
      <label>Workers (AUTOMATIC)<input name="worker_size" type="number" value="1"></label></div>
    <div class="row"><label>Network<select name="network_plugin">${(plan.networks || []).map((n) => `<option>${esc(n.name)}</option>`).join("")}</select></label>
      <label>Storage<select name="persistent_storage">${(plan.storages || []).map((s) => `<option>${esc(s.name)}</option>`).join("")}</select></label>
      <label>Domain suffix<input name="cluster_doamin_suffix" value="cluster.local"></label></div>
    <label><input type="checkbox" name="gpu_install" style="width:auto" checked> Install ROCm + AMD device plugin on GPU nodes</label>
    <h3>Nodes (MANUAL)</h3><div id="nodes"></div>
    <div id="checks"></div>
    <div class="toolbar"><button type="submit">Create</button><button type="button" id="cc-install" class="secondary">Create &amp; install</button></div>
    <p class="error" id="cc-err"></p></form>`;
  const form = $("#cc");
  const renderNodes = () => {
    const t = tmpls.find((x) => x.name === form.template.value) || {roles: []};
    const roles = (t.roles || []).map((r) => r.name);
    $("#nodes").innerHTML = table(free, [["Host", "name"], ["IP", "ip"], ["CPU", "cpu_core"], ["Mem MiB", "memory"], ["GPUs", (h) => `${h.gpu_num || 0} ${esc(h.gpu_info || "")}`],
      ["Role", (h) => `<select data-host="${esc(h.name)}"><option value="">(not used)</option>${roles.map((r) => `<option>${esc(r)}</option>`).join("")}</select>`]], "No free hosts: register hosts first.");
    $("#nodes").querySelectorAll("select").forEach((s) => s.onchange = checkDevices);
  };
  // device checks against template meta.requires (device-check.service.ts)
  const checkDevices = () => {
    const t = tmpls.find((x) => x.name === form.template.value) || {};
    const msgs = [];
    const counts = {};
    $("#nodes").querySelectorAll("select").forEach((s) => {
      if (!s.value) return;
      counts[s.value] = (counts[s.value] || 0) + 1;
      const h = free.find((x) => x.name === s.dataset.host);
      const req = ((t.roles || []).find((r) => r.name === s.value) || {}).meta?.requires || {};
      for (const d of req.device_require || []) {
        const have = d.name === "memory_size" ? (h.memory || 0) / 1024 : (h[d.name] || 0);
        if (have < d.minimal) msgs.push(`${h.name}: ${d.verbose} ${have.toFixed ? have.toFixed(0) : have} < ${d.minimal} ${d.unit || ""}`);
      }
    });
    for (const r of t.roles || []) {
      const need = r.meta?.requires?.nodes_require;
      if (!Array.isArray(need) || r.meta?.hidden) continue;
      const n = counts[r.name] || 0, [op, k] = need;
      // ">" means "at least k" as in the reference wizard (cluster-create.component.ts:307-312 opens k node slots)
      const ok = op === "=" ? n === k : (op === ">=" || op === ">") ? n >= k : true;
      if (!ok) msgs.push(`role ${r.name}: needs ${op} ${k} node(s), selected ${n}`);
    }
    $("#checks").innerHTML = msgs.length ? `<p class="error">${msgs.map(esc).join("<br>")}</p>` : "";
  };
  form.template.onchange = renderNodes;
  renderNodes();
  const submit = async (install) => {
    const f = new FormData(form);
    const d = Object.fromEntries(f.entries());
    d.configs = {gpu_install: !!form.gpu_install.checked};
    delete d.gpu_install;
    d.worker_size = Number(d.worker_size || 1);
    if (!d.plan) delete d.plan;
    d.nodes = [];
    $("#nodes").querySelectorAll("select").forEach((s) => { if (s.value) d.nodes.push({name: s.dataset.host, host: s.dataset.host, roles: [s.value]}); });
    try {
      const c = await POST("/clusters/", d);
      if (install) await POST(`/clusters/${c.name}/executions/`, {operation: "install", params: {}});
      location.hash = `#/cluster/${c.name}/${install ? "deploy" : "overview"}`;
    } catch (e) { $("#cc-err").textContent = e.message; }
  };
  form.addEventListener("submit", (e) => { e.preventDefault(); submit(false); });
  $("#cc-install").onclick = () => submit(true);
};

const OPS = [["install", "Install"], ["gpu-validate", "Validate GPUs"], ["app-deploy", "Deploy app"], ["upgrade", "Upgrade"], ["scale", "Scale (IaaS)"],
  ["add-worker", "Add worker"], ["remove-worker", "Remove worker"], ["backup", "Backup"], ["restore", "Restore"],
  ["bigip-config", "F5 BIG-IP"], ["uninstall", "Uninstall"]];

async function runOp(c, op) {
  const params = {};
  const go = async (p) => { const e = await POST(`/clusters/${c.name}/executions/`, {operation: op, params: p}); location.hash = `#/cluster/${c.name}/deploy/${e.id}`; };
  if (op === "upgrade") {
    const pk = await GET("/packages/");
    return formModal("Upgrade", [["package", "Package", "select", pk.map((p) => p.name)]], (d) => go(d));
  }
  if (op === "scale") return formModal("Scale workers", [["num", "Worker count", "number", c.worker_size]], (d) => go(d));
  if (op === "add-worker") {
    const hosts = (await GET("/host/")).filter((h) => !h.node_id);
    return formModal("Add worker", [["host", "Host", "select", hosts.map((h) => h.name)]], (d) => go(d));
  }
  if (op === "remove-worker") {
    const nodes = (await GET(`/clusters/${c.name}/nodes/`)).filter((n) => (n.roles || []).includes("worker") || (n.groups || []).includes("worker"));
    return formModal("Remove worker", [["node", "Node", "select", nodes.map((n) => n.name)]], (d) => go(d));
  }
  if (op === "backup") {
    const s = await GET("/backupStorage/");
    return formModal("Backup", [["backupStorageId", "Storage", "select", s.map((x) => [x.id, x.name])]], (d) => go(d));
  }
  if (op === "restore") {
    const b = await GET(`/clusterBackup/${c.project_id}/`);
    return formModal("Restore", [["clusterBackupId", "Backup", "select", b.map((x) => [x.id, x.name])]], (d) => go(d));
  }
  if (op === "app-deploy") { location.hash = `#/cluster/${c.name}/apps`; return; }
  if (!confirm(`${op} cluster ${c.name}?`)) return;
  await go(params);
}

let liveSockets = [];
function closeSockets() { liveSockets.forEach((s) => { try { s.close(); } catch { /* ignore */ } }); liveSockets = []; }

views.cluster = async (v, [name, tab = "overview", arg]) => {
  const c = await GET(`/clusters/${name}/`);
  const tabs = ["overview", "nodes", "deploy", "apps", "health", "events", "storage", "backup", "grade", "configs", "f5", "terminal"];
  v.innerHTML = `<h2>${esc(c.name)} ${st(c.status)}</h2><div class="tabs">${tabs.map((t) => `<a href="#/cluster/${esc(name)}/${t}" class="${t === tab ? "active" : ""}">${t}</a>`).join("")}</div><div id="tab"></div>`;
  const t = $("#tab");
  if (tab === "overview") {
    t.innerHTML = `<div class="toolbar">${OPS.map(([op, label]) => `<button class="${op === "uninstall" ? "" : "secondary"}" data-op="${op}">${label}</button>`).join("")}
      <a href="${API}/cluster/${esc(c.name)}/download/" id="kc">kubeconfig</a></div>${kv({template: c.template, package: c.package, network: c.network_plugin,
      storage: c.persistent_storage, deploy_type: c.deploy_type, nodes: c.node_size, gpus: c.gpu_num, domain: c.cluster_doamin_suffix, item: c.item_name,
      created: c.date_created, last_operation: c.current_execution ? `${c.current_execution.operation} ${c.current_execution.state}` : "—"})}`;
    t.querySelectorAll("[data-op]").forEach((b) => b.onclick = () => runOp(c, b.dataset.op).catch((e) => alert(e.message)));
    $("#kc").onclick = async (e) => { e.preventDefault(); const r = await api("GET", `/cluster/${c.name}/download/`, undefined, {raw: true}); const blob = await r.blob();
      const a = document.createElement("a"); a.href = URL.createObjectURL(blob); a.download = `${c.name}-kubeconfig`; a.click(); };
  } else if (tab === "nodes") {
    const nodes = await GET(`/clusters/${name}/nodes/`);
    t.innerHTML = table(nodes, [["Name", "name"], ["IP", "ip"], ["Roles", (n) => esc((n.roles || n.groups || []).join(", "))], ["GPUs", (n) => esc((n.vars || {}).gpu_num || 0)],
      ["Conditions", (n) => (n.conditions || []).map((x) => st(`${x.type}:${x.status}`)).join(" ")]]);
  } else if (tab === "deploy") {
    const execs = await GET(`/clusters/${name}/executions/`);
    const cur = arg || (execs[0] && execs[0].id);
    t.innerHTML = `<div class="row"><div style="flex:0 0 320px">${table(execs, [["Operation", (e) => `<a href="#/cluster/${esc(name)}/deploy/${esc(e.id)}">${esc(e.operation)}</a>`],
      ["State", (e) => st(e.state)], ["Time", (e) => `${(e.timedelta || 0).toFixed(1)}s`]])}</div>
      <div><div id="steps" class="steps"></div><pre class="term" id="term"></pre><div id="trace"></div></div></div>`;
    if (cur) follow(cur, name, t);
  } else if (tab === "health") {
    const [h, hist, comps, nss] = await Promise.all([GET(`/cluster/${name}/health/all/`).catch((e) => ({error: e.message})), GET(`/clusterHealthHistory/${c.project_id}/`).catch(() => []),
      GET(`/cluster/${name}/component/`).catch(() => []), GET(`/cluster/${name}/namespace/`).catch(() => [])]);
    t.innerHTML = `<div class="toolbar"><button id="chk" class="secondary">Check nodes</button><button id="tsk" class="secondary">Check node clocks</button></div><div id="hx"></div>` +
      (h.error ? `<p class="muted">${esc(h.error)}</p>` : kv(h)) +
      `<h3>Control-plane components (kube-system)</h3>${table(comps, [["Name", "name"], ["Ready", (d) => `${esc(d.ready_replicas ?? d.ready ?? "")}/${esc(d.replicas ?? "")}`], ["Status", (d) => st(d.status || "")]], "No data.")}
       <h3>Namespaces</h3>${table(nss, [["Name", "name"], ["Status", (n) => st(n.status)]], "No data.")}
       <h3>Availability history</h3>${table(hist, [["Date", "date_created"], ["Rate", "available_rate"], ["Type", "date_type"]])}`;
    $("#chk").onclick = async () => { const r = await GET(`/cluster/${name}/checkNodes/`).catch((e) => ({error: e.message})); $("#hx").innerHTML = r.error ? `<p class="error">${esc(r.error)}</p>` :
      table(Array.isArray(r) ? r : (r.nodes || []), [["Node", "name"], ["Conditions", (n) => (n.conditions || []).map((x) => st(`${x.type}:${x.status}`)).join(" ")]]); };
    $("#tsk").onclick = async () => { const r = await GET(`/cluster/${name}/syncNodeTime/`).catch((e) => ({error: e.message})); $("#hx").innerHTML = r.error ? `<p class="error">${esc(r.error)}</p>` : kv(r); };
  } else if (tab === "events") {
    const ev = await POST(`/cluster/${name}/event/`, {limit: 200}).catch((e) => ({items: [], error: e.message}));
    t.innerHTML = table(ev.items || ev, [["Time", "last_timestamp"], ["Type", (e) => st(e.type)], ["Reason", "reason"], ["Object", "name"], ["Message", "message"]], ev.error || "No events.");
  } else if (tab === "backup") {
    const [bks, strat, stores] = await Promise.all([GET(`/clusterBackup/${c.project_id}/`), GET("/backupStrategy/"), GET("/backupStorage/")]);
    const mine = strat.find((s) => s.cluster_id === c.id);
    t.innerHTML = `<h3>Strategy</h3>${mine ? kv(mine) : "<p class='muted'>none</p>"}<div class="toolbar"><button id="strat" class="secondary">Set strategy</button></div>
      <h3>Backups</h3>${table(bks, [["Name", "name"], ["Size", "size"], ["Date", "date_created"], ["", (b) => `<button class="link" data-restore="${esc(b.id)}">restore</button><button class="link" data-del="${esc(b.id)}">delete</button>`]])}`;
    $("#strat").onclick = () => formModal("Backup strategy", [["backup_storage_id", "Storage", "select", stores.map((s) => [s.id, s.name])], ["cron", "Every N days", "number", 1],
      ["save_num", "Keep", "number", 7], ["status", "Status", "select", ["ENABLE", "DISABLE"]]],
      (d) => mine ? PATCH(`/backupStrategy/${mine.id}/`, d) : POST("/backupStrategy/", {...d, cluster_id: c.id}), mine || {});
    t.querySelectorAll("[data-restore]").forEach((b) => b.onclick = () => confirmDo("Restore this backup?", () => POST("/clusterBackup/restore/", {id: b.dataset.restore})));
    t.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo("Delete backup?", () => DEL(`/clusterBackup/${b.dataset.del}/delete/`)));
  } else if (tab === "grade") {
    const g = await GET(`/cluster/${name}/grade/`).catch((e) => ({error: e.message}));
    t.innerHTML = g.error ? `<p class="muted">${esc(g.error)}</p>` : `<div class="grid"><div class="card stat"><div class="v">${g.score}</div><div class="k">score</div></div></div>` +
      table(g.results, [["Namespace", "namespace"], ["Workload", "name"], ["Container", "container"], ["Findings", (r) => r.results.filter((x) => !x.success).map((x) => st(x.id)).join(" ")]]);
  } else if (tab === "configs") {
    const cfgs = await GET(`/clusters/${name}/configs/`);
    t.innerHTML = `<div class="toolbar"><button id="addcfg">Set</button></div>` + table(cfgs, [["Key", "key"], ["Value", (x) => esc(JSON.stringify(x.value))], ["", (x) => `<button class="link" data-del="${esc(x.key)}">delete</button>`]]);
    $("#addcfg").onclick = () => formModal("Set config", [["key", "Key"], ["value", "Value (JSON)", "text"]], (d) => {
      let val = d.value; try { val = JSON.parse(d.value); } catch { /* keep string */ }
      return POST(`/clusters/${name}/configs/`, {key: d.key, value: val}); });
    t.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo("Delete config?", () => DEL(`/clusters/${name}/configs/${b.dataset.del}/`)));
  } else if (tab === "apps") {
    // Helm releases (app-deploy / app-remove executions) + the add-on links of the plan
    const [rel, cat] = await Promise.all([GET(`/clusters/${name}/apps/`), GET("/apps/catalog/")]);
    t.innerHTML = `<div class="toolbar"><button id="deployapp">Deploy application</button></div>
      <h3>Releases</h3>${table(rel, [["Release", "release"], ["Namespace", "namespace"], ["Chart", "chart"], ["Deployed", "date"],
        ["Result", (a) => a.training ? `${Math.round(a.training.tokens_per_s).toLocaleString()} tokens/s · ${esc(a.training.step_s)} s/step · loss ${esc(a.training.loss)}` : ""],
        ["", (a) => `<a href="#/cluster/${esc(name)}/deploy/${esc(a.execution_id)}">log</a> <button class="link" data-rm="${esc(a.release)}" data-ns="${esc(a.namespace)}">remove</button>`]], "No applications deployed.")}
      <h3>Add-on consoles</h3>${table(c.apps || [], [["App", "name"], ["URL", (a) => `<a href="${esc(a.url)}" target="_blank">${esc(a.url)}</a>`], ["Description", "describe"]])}`;
    $("#deployapp").onclick = () => {
      modal(`<h2>Deploy application</h2><form id="af"><label>Chart<select name="chart">${cat.map((x) => `<option value="${esc(x.name)}">${esc(x.name)} ${esc(x.version)} — ${esc(x.description)}</option>`).join("")}</select></label>
        <div class="row"><label>Release<input name="release" placeholder="(chart name)"></label><label>Namespace<input name="namespace" value="default"></label></div>
        <label>Values (JSON, chart defaults shown)<textarea name="values" style="min-height:260px"></textarea></label>
        <label><input type="checkbox" name="wait_job" style="width:auto"> Wait for the Job to finish and collect its result (training chart)</label>
        <div class="toolbar"><button type="submit">Deploy</button><button type="button" class="secondary" onclick="closeModal()">Cancel</button></div><p class="error" id="af-err"></p></form>`);
      const f = $("#af");
      const fill = () => { const x = cat.find((y) => y.name === f.chart.value); f.values.value = JSON.stringify(x ? x.values : {}, null, 2); f.wait_job.checked = f.chart.value === "pytorch-rocm-train"; };
      f.chart.onchange = fill; fill();
      f.addEventListener("submit", async (e) => {
        e.preventDefault();
        let values; try { values = JSON.parse(f.values.value || "{}"); } catch (err) { $("#af-err").textContent = err.message; return; }
        const params = {chart: f.chart.value, namespace: f.namespace.value || "default", values, wait_job: f.wait_job.checked};
        if (f.release.value) params.release = f.release.value;
        try { const ex = await POST(`/clusters/${name}/executions/`, {operation: "app-deploy", params}); closeModal(); location.hash = `#/cluster/${name}/deploy/${ex.id}`; }
        catch (err) { $("#af-err").textContent = err.message; }
      });
    };
    t.querySelectorAll("[data-rm]").forEach((b) => b.onclick = () => confirmDo(`Remove release ${b.dataset.rm}?`, async () => {
      const ex = await POST(`/clusters/${name}/executions/`, {operation: "app-remove", params: {release: b.dataset.rm, namespace: b.dataset.ns}});
      location.hash = `#/cluster/${name}/deploy/${ex.id}`; }));
  } else if (tab === "storage") {
    const d = await GET(`/cluster/${name}/storage/`).catch((e) => ({error: e.message}));
    t.innerHTML = d.error ? `<p class="muted">${esc(d.error)}</p>` :
      `<h3>Storage classes</h3>${table(d.storage_classes, [["Name", (x) => esc(x.metadata.name)], ["Provisioner", "provisioner"], ["Reclaim", "reclaimPolicy"],
        ["Default", (x) => ((x.metadata.annotations || {})["storageclass.kubernetes.io/is-default-class"] === "true" ? "yes" : "")]])}
       <h3>Persistent volume claims</h3>${table(d.pvcs, [["Namespace", (x) => esc(x.metadata.namespace)], ["Name", (x) => esc(x.metadata.name)],
        ["Class", (x) => esc(x.spec.storageClassName)], ["Size", (x) => esc(((x.spec.resources || {}).requests || {}).storage)], ["Phase", (x) => st((x.status || {}).phase)]])}`;
  } else if (tab === "f5") {
    const cfgs = Object.fromEntries((await GET(`/clusters/${name}/configs/`)).map((x) => [x.key, x.value]));
    // the variables of roles/f5 (k8s-bigip-ctlr --bigip-url, credentials secret, virtual-server address)
    const keys = [["bigip_url", "BIG-IP URL (https://host[:port])"], ["bigip_user", "User"], ["bigip_password", "Password"], ["bigip_partition", "Partition"], ["public_ip", "Virtual server IP"]];
    t.innerHTML = `<form id="f5" class="card">${keys.map(([k, l]) => `<label>${esc(l)}<input name="${k}" type="${k.includes("password") ? "password" : "text"}" value="${esc(k.includes("password") ? "" : (cfgs[k] ?? ""))}"></label>`).join("")}
      <div class="toolbar"><button type="submit">Save &amp; configure F5</button></div><p class="error" id="f5-err"></p></form>`;
    $("#f5").addEventListener("submit", async (e) => {
      e.preventDefault();
      try {
        for (const [k] of keys) { const v = e.target.elements[k].value; if (v !== "" || !k.includes("password")) await POST(`/clusters/${name}/configs/`, {key: k, value: v}); }
        const ex = await POST(`/clusters/${name}/executions/`, {operation: "bigip-config", params: {}});
        location.hash = `#/cluster/${name}/deploy/${ex.id}`;
      } catch (err) { $("#f5-err").textContent = err.message; }
    });
  } else if (tab === "terminal") {
    t.innerHTML = `<p class="muted">Web terminal (webkubectl) with this cluster's kubeconfig.</p><div class="toolbar"><button id="wk">Open terminal</button>
      <button id="tok" class="secondary">Show service-account token</button></div><pre class="term" id="wk-out" style="height:auto;min-height:60px"></pre>`;
    $("#wk").onclick = async () => { try { const r = await GET(`/cluster/${c.name}/webkubectl/token/`); window.open(`/webkubectl/terminal/?token=${encodeURIComponent(r.token)}`, "_blank"); }
      catch (e) { $("#wk-out").textContent = e.message; } };
    $("#tok").onclick = async () => { try { $("#wk-out").textContent = (await GET(`/cluster/${c.name}/token/`)).token; } catch (e) { $("#wk-out").textContent = e.message; } };
  }
};

// Where an execution's time went: per step, its slowest tasks (span trace summary), and the full trace as
// Chrome trace-event JSON for Perfetto / chrome://tracing.
async function showTrace(name, eid) {
  const box = $("#trace");
  if (!box || box.dataset.eid === eid) return;
  box.dataset.eid = eid;
  const sm = await GET(`/clusters/${name}/executions/${eid}/trace/?view=summary`).catch(() => null);
  if (!sm) { box.innerHTML = ""; return; }
  box.innerHTML = `<h3>Time breakdown (${sm.total_seconds.toFixed(1)} s) <button class="link" id="dltrace">download trace</button></h3>` +
    sm.steps.map((s) => `<h4>${esc(s.step)} — ${s.seconds.toFixed(1)} s, ${s.task_count} tasks ${st(s.status)}</h4>` +
      table(s.tasks, [["Slowest tasks", "task"], ["Seconds", (x) => x.seconds.toFixed(2)], ["Hosts", "hosts"],
        ["Slowest host", (x) => x.slowest_host ? `${esc(x.slowest_host)} (${x.slowest_host_seconds.toFixed(2)} s)` : ""]])).join("");
  $("#dltrace").onclick = async () => {
    const tr = await GET(`/clusters/${name}/executions/${eid}/trace/`);
    const a = document.createElement("a");
    a.href = URL.createObjectURL(new Blob([JSON.stringify(tr)], {type: "application/json"}));
    a.download = `execution-${eid}.trace.json`; a.click(); URL.revokeObjectURL(a.href);
  };
}

function follow(eid, name, root) {
  // a render that lost the race to a newer one (its tab is no longer in the page) opens no sockets
  if (root && $("#tab") !== root) return;
  closeSockets();
  const term = (root || document).querySelector("#term"), steps = (root || document).querySelector("#steps");
  const tok = localStorage.getItem("kop_token");
  const p = new WebSocket(wsURL(`/ws/progress/${eid}/?token=${encodeURIComponent(tok)}`));
  p.onmessage = (m) => { const d = JSON.parse(m.data); steps.innerHTML = (d.steps || []).map((s) => `<span class="${esc(s.status)}">${esc(s.name)}</span>`).join("") + ` ${st(d.state)}`;
    if (name && (d.state === "SUCCESS" || d.state === "FAILURE")) showTrace(name, eid); };
  const l = new WebSocket(wsURL(`/ws/tasks/${eid}/log/?token=${encodeURIComponent(tok)}`));
  l.onmessage = (m) => { term.textContent += JSON.parse(m.data).message.replace(/\r\n/g, "\n"); term.scrollTop = term.scrollHeight; };
  liveSockets.push(p, l);
}

views.hosts = async (v) => {
  const [rows, creds, zones] = await Promise.all([GET("/host/"), GET("/credential/"), GET("/zones/")]);
  v.innerHTML = `<h2>Hosts</h2><div class="toolbar"><button id="add">Register host</button><label class="secondary" style="margin:0">Import (.xlsx/.csv)
    <input type="file" id="imp" accept=".xlsx,.csv" style="width:auto"></label></div>
    ${table(rows, [["Name", "name"], ["IP", "ip"], ["Status", (h) => st(h.status)], ["OS", (h) => `${esc(h.os)} ${esc(h.os_version)}`], ["CPU", "cpu_core"], ["Mem MiB", "memory"],
      ["GPUs", (h) => h.gpu_num ? `${h.gpu_num} × ${esc(h.gpu_info)}` : "—"], ["Cluster", (h) => h.node_id ? "in use" : ""],
      ["", (h) => `<button class="link" data-sync="${esc(h.id)}">sync</button><button class="link" data-del="${esc(h.id)}">delete</button>`]])}`;
  $("#add").onclick = () => formModal("Register host", [["name", "Name"], ["ip", "IP"], ["port", "SSH port", "number", 22], ["credential", "Credential", "select", [["", "(username/password below)"], ...creds.map((c) => [c.id, c.name])]],
    ["username", "Username", "text", "root"], ["password", "Password", "password"], ["zone_id", "Zone", "select", [["", "—"], ...zones.map((z) => [z.id, z.name])]]],
    (d) => { if (!d.credential) delete d.credential; if (!d.zone_id) delete d.zone_id; return POST("/host/", d); });
  $("#imp").onchange = async (e) => { const fd = new FormData(); fd.append("file", e.target.files[0]); try { const r = await api("POST", "/host/import/", fd); alert(`created: ${r.created.join(", ")}\n${(r.errors || []).join("\n")}`); route(); } catch (err) { alert(err.message); } };
  v.querySelectorAll("[data-sync]").forEach((b) => b.onclick = () => POST(`/host/${b.dataset.sync}/sync/`).then(() => setTimeout(route, 1500)));
  v.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo("Delete host?", () => DEL(`/host/${b.dataset.del}/`)));
};

views.credentials = crudPage("Credentials", "/credential/", [["Name", "name"], ["Username", "username"], ["Type", "type"]],
  [["name", "Name"], ["username", "Username", "text", "root"], ["type", "Type", "select", ["password", "privateKey"]], ["password", "Password", "password"], ["private_key", "Private key", "textarea"]]);

views.packages = async (v) => {
  const rows = await GET("/packages/");
  v.innerHTML = `<h2>Offline packages</h2>${table(rows, [["Name", "name"], ["Version", (p) => esc(p.meta.version)], ["Kubernetes", (p) => esc((p.meta.vars || {}).kube_version)],
    ["ROCm", (p) => esc((p.meta.vars || {}).rocm_version)], ["AMD device plugin", (p) => esc((p.meta.vars || {}).amd_device_plugin_image || "")],
    ["Repository", (p) => endpoint(p, "repo", p.repo_port, "/repository/")], ["Registry", (p) => endpoint(p, "registry", p.registry_port, "/v2/")],
    ["Path", "path"]])}`;
};
// a package endpoint: port and whether the repo service serves it (or why not: a port claimed by another package)
function endpoint(p, kind, port, path) {
  if (p.conflict) return `<span class="bad" title="${esc(p.conflict)}">:${esc(port)} refused</span>`;
  const on = (p.serving || {})[kind];
  return on ? `<span class="ok">:${esc(port)}${esc(path)}</span>` : `<span class="muted">:${esc(port)} (no content)</span>`;
}

views.regions = crudPage("Regions", "/regions/", [["Name", "name"], ["Cloud region", "cloud_region"], ["Provider", (r) => esc((r.vars || {}).provider || "")]],
  [["name", "Name"], ["cloud_region", "Cloud region"], ["template_id", "Provider template id"], ["vars", "Provider vars (JSON: provider, host/user/password …)", "json"], ["comment", "Comment"]]);
views.zones = crudPage("Zones", "/zones/", [["Name", "name"], ["Cloud zone", "cloud_zone"], ["IP range", (z) => esc(`${(z.vars || {}).ip_start || ""} – ${(z.vars || {}).ip_end || ""}`)],
  ["Used IPs", (z) => (z.ip_used || []).length], ["Status", (z) => st(z.status)]],
  [["name", "Name"], ["region_id", "Region id"], ["cloud_zone", "Cloud zone"], ["vars", "Zone vars (JSON: ip_start, ip_end, net_mask, gateway, dns1 …)", "json"]]);
views.plans = crudPage("Deploy plans", "/plans/", [["Name", "name"], ["Template", "deploy_template"], ["Zones", (p) => (p.zone_ids || []).length], ["Compute", (p) => esc(JSON.stringify(p.vars || {}))]],
  [["name", "Name"], ["region_id", "Region id"], ["zone_ids", "Zone ids (JSON list)", "json"], ["deploy_template", "Template", "select", ["SINGLE", "MULTIPLE"]],
   ["vars", "Vars (JSON: master_model, worker_model, gpu_worker …)", "json"]]);

views.storage = async (v) => {
  const [nfs, ceph] = await Promise.all([GET("/storage/nfs/"), GET("/storage/ceph/")]);
  v.innerHTML = `<h2>Storage</h2><h3>NFS</h3><div class="toolbar"><button id="nfs">Add NFS</button></div>
    ${table(nfs, [["Name", "name"], ["Server", (n) => esc((n.vars || {}).storage_nfs_server)], ["Path", (n) => esc((n.vars || {}).storage_nfs_server_path)], ["Status", (n) => st(n.status)],
      ["", (n) => `<button class="link" data-dn="${esc(n.name)}">delete</button>`]])}
    <h3>Ceph</h3><div class="toolbar"><button id="ceph">Add Ceph</button></div>${table(ceph, [["Name", "name"], ["Monitors", (c) => esc((c.vars || {}).monitors)],
      ["", (c) => `<button class="link" data-dc="${esc(c.name)}">delete</button>`]])}`;
  $("#nfs").onclick = () => formModal("NFS", [["name", "Name"], ["vars", "Vars (JSON: storage_nfs_server, storage_nfs_server_path, external, username, password)", "json"]], (d) => POST("/storage/nfs/", d));
  $("#ceph").onclick = () => formModal("Ceph", [["name", "Name"], ["vars", "Vars (JSON: monitors, pool, user, key)", "json"]], (d) => POST("/storage/ceph/", d));
  v.querySelectorAll("[data-dn]").forEach((b) => b.onclick = () => confirmDo("Delete?", () => DEL(`/storage/nfs/${b.dataset.dn}/`)));
  v.querySelectorAll("[data-dc]").forEach((b) => b.onclick = () => confirmDo("Delete?", () => DEL(`/storage/ceph/${b.dataset.dc}/`)));
};

views.items = async (v) => {
  const [items, users] = await Promise.all([GET("/items/"), GET("/users/")]);
  v.innerHTML = `<h2>Items (projects)</h2><div class="toolbar"><button id="add">Add item</button></div>
    ${table(items, [["Name", "name"], ["Description", "description"], ["", (i) => `<button class="link" data-mem="${esc(i.name)}">members</button><button class="link" data-res="${esc(i.name)}">resources</button><button class="link" data-del="${esc(i.id)}">delete</button>`]])}
    <div id="detail"></div>`;
  $("#add").onclick = () => formModal("Item", [["name", "Name"], ["description", "Description"]], (d) => POST("/items/", d));
  v.querySelectorAll("[data-del]").forEach((b) => b.onclick = () => confirmDo("Delete item?", () => DEL(`/items/${b.dataset.del}/`)));
  v.querySelectorAll("[data-mem]").forEach((b) => b.onclick = async () => {
    const mem = await GET(`/item/profiles/${b.dataset.mem}/`);
    $("#detail").innerHTML = `<h3>Members of ${esc(b.dataset.mem)}</h3>${table(mem, [["User", "username"], ["Role", "role"]])}<div class="toolbar"><button id="setm" class="secondary">Edit members</button></div>`;
    $("#setm").onclick = () => formModal("Members", [["profiles", "JSON list of {username, role: VIEWER|MANAGER}", "json"]],
      (d) => POST(`/item/profiles/${b.dataset.mem}/`, d.profiles), {profiles: mem.map((m) => ({username: m.username, role: m.role}))});
  });
  v.querySelectorAll("[data-res]").forEach((b) => b.onclick = async () => {
    const res = await GET(`/resource/${b.dataset.res}/`);
    $("#detail").innerHTML = `<h3>Resources of ${esc(b.dataset.res)}</h3>${table(res, [["Type", "resource_type"], ["Id", "resource_id"]])}
      <div class="toolbar"><button id="addr" class="secondary">Add resources</button></div>`;
    $("#addr").onclick = () => formModal("Add resources", [["type", "Type", "select", ["CLUSTER", "HOST", "PLAN", "BACKUP_STORAGE", "STORAGE"]], ["ids", "Ids (JSON list)", "json"]],
      (d) => POST(`/resource/${b.dataset.res}/${d.type}/`, d.ids));
  });
  void users;
};

views.users = crudPage("Users", "/users/", [["Username", "username"], ["Email", "email"], ["Superuser", "is_superuser"], ["Active", "is_active"], ["Source", "source"]],
  [["username", "Username"], ["email", "Email"], ["password", "Password", "password"], ["is_superuser", "Superuser", "checkbox"], ["is_active", "Active", "checkbox", true]],
  {extraButtons: `<button class="secondary" onclick="POST('/users/sync/').then(()=>alert('LDAP sync queued'))">Sync LDAP</button>`});

views.settings = async (v, [tab = "system"]) => {
  const tabs = ["system", "dns", "backup-storage", "ldap", "notification"];
  v.innerHTML = `<h2>Settings</h2><div class="tabs">${tabs.map((t) => `<a href="#/settings/${t}" class="${t === tab ? "active" : ""}">${t}</a>`).join("")}</div><div id="tab"></div>`;
  const t = $("#tab");
  if (tab === "backup-storage") return crudPage("Backup storage", "/backupStorage/", [["Name", "name"], ["Type", "type"], ["Region", "region"], ["Status", (b) => st(b.status)]],
    [["name", "Name"], ["type", "Type", "select", ["S3", "OSS", "AZURE", "LOCAL"]], ["region", "Region"], ["credentials", "Credentials (JSON: bucket, accessKey, secretKey, endpoint | path)", "json"]])(t);
  if (tab === "dns") {  // cluster-wide node resolvers (the reference's DNS page): /dns/, /dns/update/
    const d = await GET("/dns/");
    t.innerHTML = `<form id="df" class="card"><label>DNS1<input name="dns1" value="${esc(d.dns1)}"></label><label>DNS2<input name="dns2" value="${esc(d.dns2)}"></label>
      <div class="toolbar"><button type="submit">Save</button></div><p id="df-msg" class="muted">Written to every node's resolv.conf at install; a zone's own dns1 / dns2 take precedence.</p></form>`;
    $("#df").addEventListener("submit", async (e) => {
      e.preventDefault();
      const f = new FormData(e.target);
      try {
        await POST("/dns/update/", {dns1: f.get("dns1"), dns2: f.get("dns2")});
        $("#df-msg").textContent = "Saved.";
      } catch (err) { $("#df-msg").textContent = String(err.message || err); }
    });
    return;
  }
  const keys = {system: ["local_hostname", "domain_suffix", "ntp_server", "REGISTRY_PREFIX"], ldap: ["AUTH_LDAP_ENABLE", "AUTH_LDAP_SERVER_URI", "AUTH_LDAP_BIND_DN", "AUTH_LDAP_BIND_PASSWORD", "AUTH_LDAP_SEARCH_OU", "AUTH_LDAP_SEARCH_FILTER", "AUTH_LDAP_USER_ATTR_MAP"],
    notification: ["SMTP_ADDRESS", "SMTP_PORT", "SMTP_USERNAME", "SMTP_PASSWORD", "SMTP_USE_SSL", "DINGTALK_WEBHOOK", "DINGTALK_SECRET", "WORKWEIXIN_CORP_ID", "WORKWEIXIN_AGENT_ID", "WORKWEIXIN_SECRET"]}[tab];
  const cur = await GET(`/settings?tab=${tab}`);
  t.innerHTML = `<form id="sf" class="card">${keys.map((k) => `<label>${esc(k)}<input name="${k}" type="${/PASSWORD|SECRET/.test(k) ? "password" : "text"}" value="${esc(cur[k] ?? "")}"></label>`).join("")}
    <div class="toolbar"><button type="submit">Save</button>${tab === "notification" ? `<button type="button" id="testmail" class="secondary">Test email</button>` : ""}</div><p id="sf-msg" class="muted"></p></form>`;
  $("#sf").addEventListener("submit", async (e) => {
    e.preventDefault();
    const d = Object.fromEntries(new FormData(e.target).entries());
    for (const k of Object.keys(d)) if (/PASSWORD|SECRET/.test(k) && !d[k]) delete d[k];
    await api("POST", `/settings?tab=${tab}`, d); $("#sf-msg").textContent = "saved";
  });
  if ($("#testmail")) $("#testmail").onclick = async () => { const d = Object.fromEntries(new FormData($("#sf")).entries()); const r = await POST("/notification/email/check/", d); $("#sf-msg").textContent = r.success ? "email sent" : "email failed"; };
};

views.messages = async (v) => {
  const [ms, sub, rcv] = await Promise.all([GET("/notification/userMessage/?limit=100"), GET("/notification/subscribe/"), GET("/notification/receiver/")]);
  v.innerHTML = `<h2>Message center</h2><div class="toolbar"><button id="readall" class="secondary">Mark all read</button><button id="subs" class="secondary">Subscriptions</button><button id="rcv" class="secondary">Receivers</button></div>
    ${table(ms.results, [["", (m) => m.read_status === "UNREAD" ? "●" : ""], ["Title", (m) => esc(m.message_detail.title)], ["Level", (m) => st(m.message_detail.level)],
      ["Detail", (m) => esc(JSON.stringify(m.message_detail.content))], ["Date", "date_created"]], "No messages.")}`;
  $("#readall").onclick = () => PUT("/notification/userMessage/", {ids: null}).then(route);
  $("#subs").onclick = () => formModal("Subscriptions", [["type", "Type", "select", ["SYSTEM", "CLUSTER"]], ["vars", "Channels (JSON: LOCAL/EMAIL/DINGTALK/WORKWEIXIN: ENABLE|DISABLE)", "json"]],
    (d) => PUT("/notification/subscribe/", d), sub[0] || {vars: {LOCAL: "ENABLE", EMAIL: "DISABLE", DINGTALK: "DISABLE", WORKWEIXIN: "DISABLE"}});
  $("#rcv").onclick = () => formModal("Receivers", [["vars", "Addresses (JSON: EMAIL, DINGTALK, WORKWEIXIN)", "json"]], (d) => PUT("/notification/receiver/", d), rcv);
};

views.logs = async (v) => {
  v.innerHTML = `<h2>System log</h2><form id="lf" class="toolbar"><select name="level" style="width:auto"><option value="">any level</option><option>INFO</option><option>WARNING</option><option>ERROR</option></select>
    <input name="keywords" placeholder="keywords" style="width:260px"><input name="days" type="number" value="7" style="width:80px"><button>Search</button></form><div id="lr"></div>`;
  const run = async () => {
    const d = Object.fromEntries(new FormData($("#lf")).entries());
    const r = await POST("/log/", {...d, days: Number(d.days || 7), limit: 200});
    $("#lr").innerHTML = `<p class="muted">${r.total} entries</p>` + table(r.items, [["Time", "@timestamp"], ["Level", (x) => st(x.levelname)], ["Logger", "name"], ["Message", "msg"]]);
  };
  $("#lf").addEventListener("submit", (e) => { e.preventDefault(); run(); });
  run();
};

views.profile = async (v) => {
  v.innerHTML = `<h2>Profile</h2>${kv({username: ME.username, email: ME.email || "", superuser: ME.is_superuser, source: ME.source || "local",
    items: (ME.item_role_mappings || []).map((m) => `${m.item_name}:${m.role}`).join(", ")})}
    <h3>Change password</h3><form id="pw" class="card" style="max-width:420px"><label>Current password<input name="original" type="password"></label>
    <label>New password<input name="password" type="password"></label><label>Repeat<input name="password2" type="password"></label>
    <div class="toolbar"><button type="submit">Change</button></div><p id="pw-msg" class="muted"></p></form>`;
  $("#pw").addEventListener("submit", async (e) => {
    e.preventDefault();
    const d = Object.fromEntries(new FormData(e.target).entries());
    if (d.password !== d.password2) { $("#pw-msg").textContent = "passwords differ"; return; }
    try { await PUT("/password/", {original: d.original, password: d.password}); $("#pw-msg").textContent = "password changed"; e.target.reset(); }
    catch (err) { $("#pw-msg").textContent = err.message; }
  });
};

views.training = async (v) => {
  // the bundled PyTorch-ROCm chart: model presets and every training release across clusters
  const [presets, cls] = await Promise.all([GET("/train/presets/"), GET("/clusters/")]);
  const rels = (await Promise.all(cls.map((c) => GET(`/clusters/${c.name}/apps/`).then((r) => r.map((a) => ({...a, cluster: c.name}))).catch(() => []))))
    .flat().filter((a) => a.chart === "pytorch-rocm-train");
  v.innerHTML = `<h2>GPU training (PyTorch-ROCm chart)</h2><p class="muted">Deploy from a cluster's <i>apps</i> tab: chart <code>pytorch-rocm-train</code>, one pod per node with
    <code>amd.com/gpu</code> × gpusPerNode, torchrun over RCCL; hand-written gfx950 kernels for attention, norms, RoPE, SwiGLU, cross-entropy and AdamW.</p>
    <h3>Runs</h3>${table(rels, [["Cluster", (a) => `<a href="#/cluster/${esc(a.cluster)}/apps">${esc(a.cluster)}</a>`], ["Release", "release"], ["Model", (a) => esc((a.values || {}).model || "")],
      ["GPUs/node", (a) => esc((a.values || {}).gpusPerNode || "")], ["tokens/s", (a) => a.training ? Math.round(a.training.tokens_per_s).toLocaleString() : "—"],
      ["s/step", (a) => esc(a.training ? a.training.step_s : "")], ["TFLOP/s/GPU", (a) => esc(a.training ? a.training.tflops_per_gpu : "")], ["Date", "date"]], "No training runs yet.")}
    <h3>Model presets</h3>${table(Object.entries(presets).map(([k, p]) => ({name: k, ...p})), [["Preset", "name"], ["Parameters", (p) => `${(p.params / 1e9).toFixed(2)} B`], ["Layers", "layers"], ["Hidden", "hidden"]])}`;
};

// task monitor (the reference's Celery Flower at /flower/): workers, per-task statistics, recent jobs with
// revoke / retry and their logs, the periodic schedule
views.tasks = async (v, [state = ""]) => {
  const [workers, stats, recent, periodic] = await Promise.all([GET("/tasks/workers/"), GET("/tasks/stats/"),
    GET(`/tasks/?limit=200${state ? "&state=" + encodeURIComponent(state) : ""}`), GET("/tasks/periodic/")]);
  const secs = (x) => (x === null || x === undefined ? "" : `${Number(x).toFixed(2)} s`);
  v.innerHTML = `<h2>Task monitor</h2>
    <h3>Workers</h3>${table(workers, [["Worker", "name"], ["Online", (w) => st(w.online ? "online" : "offline")], ["Concurrency", "concurrency"],
      ["Running", (w) => (w.active || []).length], ["Processed", "processed"], ["Last seen", "last_seen"]], "No worker process has registered.")}
    <h3>Tasks</h3>${table(stats.tasks, [["Task", "task"], ["Total", "total"], ["Succeeded", (t) => t.success || 0], ["Failed", (t) => t.failure || 0],
      ["Pending", (t) => t.pending || 0], ["Running", (t) => t.started || 0], ["Avg", (t) => secs(t.runtime_avg_s)], ["Max", (t) => secs(t.runtime_max_s)]])}
    <h3>Recent jobs</h3><div class="toolbar">${["", "PENDING", "STARTED", "SUCCESS", "FAILURE", "REVOKED"].map((s) =>
      `<a href="#/tasks/${s}" class="${s === state ? "active" : ""}">${s || "all"}</a>`).join(" ")}</div>
    ${table(recent, [["Task", "name"], ["State", (j) => st(j.state)], ["Worker", "worker"], ["Created", "date_created"], ["Runtime", (j) => secs(j.runtime_s)],
      ["Error", "error"], ["", (j) => `<button class="link" data-log="${esc(j.id)}">log</button>` +
        (j.state === "PENDING" ? `<button class="link" data-revoke="${esc(j.id)}">revoke</button>` : "") +
        (["FAILURE", "REVOKED"].includes(j.state) ? `<button class="link" data-retry="${esc(j.id)}">retry</button>` : "")]], "No jobs.")}
    <h3>Periodic schedule</h3>${table(periodic, [["Name", "name"], ["Task", "task"], ["Cron", "crontab"], ["Every", (p) => p.interval_s ? `${p.interval_s} s` : ""],
      ["Enabled", "enabled"], ["Last run", "last_run"]])}
    <pre class="term hidden" id="joblog"></pre>`;
  v.querySelectorAll("[data-revoke]").forEach((b) => b.onclick = () => confirmDo("Revoke this job?", () => POST(`/tasks/${b.dataset.revoke}/revoke/`)));
  v.querySelectorAll("[data-retry]").forEach((b) => b.onclick = () => confirmDo("Run this job again?", () => POST(`/tasks/${b.dataset.retry}/retry/`)));
  v.querySelectorAll("[data-log]").forEach((b) => b.onclick = async () => {
    const r = await GET(`/tasks/${b.dataset.log}/log/`);
    const pre = $("#joblog"); pre.classList.remove("hidden"); pre.textContent = r.data;
  });
};

// ------------------------------------------------------------------ navigation
const NAV = [["Overview", [["dashboard", "Dashboard"], ["clusters", "Clusters"], ["training", "GPU training"]]],
  ["Infrastructure", [["hosts", "Hosts"], ["credentials", "Credentials"], ["regions", "Regions"], ["zones", "Zones"], ["plans", "Deploy plans"], ["packages", "Packages"], ["storage", "Storage"]]],
  ["Administration", [["items", "Items"], ["users", "Users"], ["settings", "Settings"], ["tasks", "Task monitor"], ["messages", "Messages"], ["logs", "System log"], ["profile", "Profile"]]]];

function renderNav(current) {
  $("#nav").innerHTML = NAV.map(([g, items]) => `<div class="group">${g}</div>` + items.filter(([k]) => ME.is_superuser || !["users", "settings", "credentials", "tasks"].includes(k))
    .map(([k, label]) => `<a href="#/${k}" class="${k === current ? "active" : ""}">${label}</a>`).join("")).join("");
}

async function route() {
  closeSockets();
  const parts = (location.hash.replace(/^#\/?/, "") || "dashboard").split("/").map(decodeURIComponent);
  const name = parts[0];
  renderNav(name === "cluster" || name === "cluster-create" ? "clusters" : name);
  const view = views[name] || views.dashboard;
  const v = $("#view");
  v.innerHTML = `<p class="muted">loading…</p>`;
  try { await view(v, parts.slice(1)); } catch (e) { v.innerHTML = `<p class="error">${esc(e.message)}</p>`; }
  GET("/notification/userMessage/unread/").then((r) => { $("#unread").textContent = r.unread; }).catch(() => {});
}

async function boot() {
  if (!localStorage.getItem("kop_token")) return showLogin();
  try { ME = await GET("/profile/"); } catch { return showLogin(); }
  $("#login").classList.add("hidden");
  $("#shell").classList.remove("hidden");
  $("#who").textContent = ME.username;
  GET("/version/").then((r) => { $("#version").textContent = `v${r.version} · ${r.accelerator}`; });
  route();
}
window.addEventListener("hashchange", route);
setInterval(refreshToken, 30 * 60 * 1000);
boot();
