// Behavioural test of the web UI against a LIVE control plane (tests/test_ui_flows.py starts it on the simulated
// farm): the real index.html + app.js run in a vm context over tests/ui/dom.js, with fetch over node's http module
// and a minimal RFC 6455 WebSocket client, and drive the reference's main flows:
//   sign in -> cluster-create wizard with device / node-count checks against the template's requires
//   (reference cluster-create.component.ts:394-505) -> create & install -> deploy tab following the progress and
//   log websockets (reference deploy/component/term/term.component.ts:54-59) until SUCCESS, with the time
//   breakdown -> apps tab: deploy the PyTorch-ROCm training chart and see its tokens/s result -> Day 2: register a
//   host through its form, add it as a worker, create a backup storage and back the cluster up, save LDAP settings,
//   add a user -> task monitor.
// Usage: node --harmony-nullish --harmony-optional-chaining tests/ui/flows.js http://127.0.0.1:PORT PASSWORD [BACKUP_DIR]
"use strict";
const http = require("http");
const crypto = require("crypto");
const vm = require("vm");
const {makeWindow, Event} = require("./dom");

const BASE = process.argv[2];
const PASSWORD = process.argv[3];
const BACKUP_DIR = process.argv[4] || "/tmp/kop-ui-backups";
const HOST = BASE.replace(/^http:\/\//, "");
const log = (step, extra) => console.log(JSON.stringify(Object.assign({step}, extra || {})));

function request(method, url, headers, body) {
  return new Promise((resolve, reject) => {
    const u = new URL(url, BASE);
    const req = http.request({method, hostname: u.hostname, port: u.port, path: u.pathname + u.search, headers: headers || {}}, (res) => {
      const chunks = [];
      res.on("data", (c) => chunks.push(c));
      res.on("end", () => resolve({status: res.statusCode, statusText: res.statusMessage, headers: res.headers, body: Buffer.concat(chunks)}));
    });
    req.on("error", reject);
    if (body !== undefined) req.write(body);
    req.end();
  });
}

async function fetchImpl(url, opts) {
  opts = opts || {};
  const r = await request(opts.method || "GET", url, opts.headers, typeof opts.body === "string" ? opts.body : undefined);
  return {
    ok: r.status >= 200 && r.status < 300, status: r.status, statusText: r.statusText,
    text: async () => r.body.toString("utf8"), json: async () => JSON.parse(r.body.toString("utf8")),
    blob: async () => ({size: r.body.length}),
  };
}

class WebSocketImpl {
  constructor(url) {
    this.readyState = 0;
    this.onmessage = null; this.onopen = null; this.onclose = null; this.onerror = null;
    const u = new URL(url);
    const key = crypto.randomBytes(16).toString("base64");
    const req = http.request({hostname: u.hostname, port: u.port, path: u.pathname + u.search, headers: {
      Connection: "Upgrade", Upgrade: "websocket", "Sec-WebSocket-Key": key, "Sec-WebSocket-Version": "13"}});
    req.on("upgrade", (res, sock) => {
      const want = crypto.createHash("sha1").update(key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11").digest("base64");
      if (res.headers["sec-websocket-accept"] !== want) { this._fail("bad Sec-WebSocket-Accept"); return; }
      this._sock = sock;
      this.readyState = 1;
      let buf = Buffer.alloc(0);
      sock.on("data", (d) => {
        buf = Buffer.concat([buf, d]);
        for (;;) {
          if (buf.length < 2) return;
          const op = buf[0] & 0x0f;
          let n = buf[1] & 0x7f, off = 2;
          if (n === 126) { if (buf.length < 4) return; n = buf.readUInt16BE(2); off = 4; }
          else if (n === 127) { if (buf.length < 10) return; n = Number(buf.readBigUInt64BE(2)); off = 10; }
          if (buf.length < off + n) return;
          const payload = buf.slice(off, off + n);
          buf = buf.slice(off + n);
          if (op === 1 && this.onmessage) this.onmessage({data: payload.toString("utf8")});
          if (op === 8) { this.readyState = 3; sock.end(); if (this.onclose) this.onclose({}); }
        }
      });
      sock.on("close", () => { this.readyState = 3; });
      if (this.onopen) this.onopen({});
    });
    req.on("response", () => this._fail("websocket upgrade refused"));
    req.on("error", (e) => this._fail(e.message));
    req.end();
  }
  _fail(msg) { this.readyState = 3; this.error = msg; if (this.onerror) this.onerror({message: msg}); }
  send() { throw new Error("the UI does not send on its websockets"); }
  close() {
    if (this._sock && this.readyState === 1) {
      const mask = crypto.randomBytes(4);
      this._sock.write(Buffer.concat([Buffer.from([0x88, 0x80]), mask]));
      this._sock.end();
    }
    this.readyState = 3;
  }
}

const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
async function until(fn, what, ms) {
  const t0 = Date.now();
  for (;;) {
    let v;
    try { v = fn(); } catch (e) { v = null; }
    if (v) return v;
    if (Date.now() - t0 > (ms || 30000)) throw new Error(`timed out waiting for ${what}`);
    await sleep(40);
  }
}

async function main() {
  const index = (await request("GET", "/ui/index.html")).body.toString();
  const app = (await request("GET", "/ui/app.js")).body.toString();
  const win = makeWindow(HOST);
  const doc = win.document;
  const body = /<body[^>]*>([\s\S]*)<\/body>/i.exec(index)[1];
  doc.body.innerHTML = body;
  const alerts = [], sockets = [], opened = [];
  const ctx = {
    window: win, document: doc, location: win.location, localStorage: win.localStorage, FormData: win.FormData,
    Event, fetch: fetchImpl, URL: {createObjectURL: () => "blob:x", revokeObjectURL: () => {}}, Blob: function Blob() {},
    WebSocket: function (url) { const s = new WebSocketImpl(url); sockets.push(s); return s; },
    alert: (m) => alerts.push(String(m)), confirm: () => true, console, setTimeout, clearTimeout,
    setInterval: () => 0, clearInterval: () => {}, encodeURIComponent, decodeURIComponent,
  };
  win.open = (u) => opened.push(u);
  vm.createContext(ctx);
  vm.runInContext(app, ctx, {filename: "app.js"});
  const $ = (s) => doc.querySelector(s);

  // ------------------------------------------------------------------ sign in
  await until(() => !$("#login").classList.contains("hidden"), "login form");
  const lf = $("#login-form");
  lf.password.value = "wrong-password";
  lf.dispatchEvent(new Event("submit", {bubbles: true}));
  await until(() => $("#login-error").textContent, "login error");
  log("login-refused", {error: $("#login-error").textContent});
  lf.password.value = PASSWORD;
  lf.dispatchEvent(new Event("submit", {bubbles: true}));
  await until(() => !$("#shell").classList.contains("hidden") && /Dashboard/.test($("#view").textContent), "dashboard");
  await until(() => $("#who").textContent === "admin", "user name");
  log("signed-in", {token: !!win.localStorage.getItem("kop_token"), nav: doc.querySelectorAll("#nav a").length});

  // ------------------------------------------------------------------ create wizard + device checks
  win.location.hash = "#/cluster-create";
  const form = await until(() => $("#cc"), "cluster-create form");
  form.name.value = "uiflow";
  form.template.value = "single-master";
  form.template.dispatchEvent(new Event("change"));
  const roleSel = (h) => doc.querySelector(`#nodes select[data-host="${h}"]`);
  await until(() => roleSel("m1") && roleSel("w1") && roleSel("tiny"), "node role selects");
  const setRole = (h, r) => { const s = roleSel(h); s.value = r; s.dispatchEvent(new Event("change")); };
  setRole("m1", "master");
  setRole("w1", "master");
  setRole("tiny", "worker");
  const checks = () => $("#checks").textContent;
  await until(() => /role master: needs = 1/.test(checks()), "node-count check");
  const failing = checks();
  if (!/tiny: Memory 2 < 8/.test(failing)) throw new Error("device check for the small host missing: " + failing);
  log("device-checks", {messages: failing});
  setRole("w1", "worker");
  setRole("tiny", "");
  await until(() => checks() === "", "checks cleared");
  log("device-checks-ok");
  form.persistent_storage.value = "local-volume";
  $("#cc-install").click();
  await until(() => win.location.hash === "#/cluster/uiflow/deploy", "navigation to the deploy tab");

  // ------------------------------------------------------------------ install, followed over the websockets
  try {
    await until(() => /SUCCESS/.test($("#steps") && $("#steps").textContent), "install SUCCESS on the progress socket", 90000);
  } catch (e) {
    log("debug", {hash: win.location.hash, view: $("#view").textContent.slice(0, 800), steps: $("#steps") && $("#steps").innerHTML,
                  sockets: sockets.map((x) => [x.readyState, x.error || ""]), alerts});
    throw e;
  }
  const steps = doc.querySelectorAll("#steps span").map((s) => [s.textContent, s.className]);
  await until(() => /Time breakdown/.test($("#trace").textContent), "time breakdown");
  await until(() => /TASK \[|PLAY/.test($("#term").textContent), "deploy log on the log socket");
  log("installed", {steps, log_bytes: $("#term").textContent.length, sockets: sockets.length,
                    socket_errors: sockets.filter((s) => s.error).map((s) => s.error)});

  // ------------------------------------------------------------------ app store: training chart
  win.location.hash = "#/cluster/uiflow/apps";
  await until(() => $("#deployapp"), "apps tab");
  $("#deployapp").click();
  const af = await until(() => $("#af"), "deploy form");
  af.chart.value = "pytorch-rocm-train";
  af.chart.dispatchEvent(new Event("change"));
  if (!af.wait_job.checked) throw new Error("the training chart should wait for its Job");
  const vals = JSON.parse(af.values.value);
  vals.gpusPerNode = 8;
  vals.steps = 20;
  af.values.value = JSON.stringify(vals);
  af.release.value = "llama-train";
  af.dispatchEvent(new Event("submit", {bubbles: true}));
  await until(() => /^#\/cluster\/uiflow\/deploy\/.+/.test(win.location.hash), "navigation to the app-deploy execution");
  await until(() => /SUCCESS/.test($("#steps").textContent), "app-deploy SUCCESS", 90000);
  win.location.hash = "#/cluster/uiflow/apps";
  const row = await until(() => doc.querySelectorAll("#tab table tr").find((r) => /llama-train/.test(r.textContent)), "release row");
  if (!/tokens\/s/.test(row.textContent)) throw new Error("no training result in the release row: " + row.textContent);
  log("app-deployed", {row: row.textContent.replace(/\s+/g, " ").trim()});
  // ------------------------------------------------------------------ Day 2: register a host through its form,
  // add it as a worker from the overview tab's operation buttons (reference cluster-status.component.ts:46-77)
  const submitModal = (fill) => { const mf = $("#mf"); fill(mf.elements); mf.dispatchEvent(new Event("submit", {bubbles: true})); };
  // an open form modal (a closed one keeps its old form in the DOM until the next one replaces it)
  const openModal = (what) => until(() => !$("#modal").classList.contains("hidden") && $("#mf"), what);
  const rowWith = (re) => doc.querySelectorAll("#view table tr").find((r) => re.test(r.textContent));
  const runOp = async (op, fill, label) => {
    win.location.hash = "#/cluster/uiflow/overview";
    const btn = await until(() => doc.querySelector(`[data-op="${op}"]`), `${op} button`);
    const before = win.location.hash;
    btn.click();
    await openModal(`${op} form`);
    submitModal(fill);
    await until(() => win.location.hash !== before && /^#\/cluster\/uiflow\/deploy\/.+/.test(win.location.hash), `${op} execution`);
    const eid = win.location.hash.split("/").pop();
    await until(() => rowWith(new RegExp(op)) && /SUCCESS/.test($("#steps").textContent), `${label} SUCCESS`, 90000);
    return eid;
  };
  win.location.hash = "#/packages";
  await until(() => rowWith(/mi355x-k8s-next.*:8083.*:8084/), "package endpoints row");
  log("package-endpoints", {row: rowWith(/mi355x-k8s-next/).textContent.replace(/\s+/g, " ").trim()});
  win.location.hash = "#/hosts";
  await until(() => $("#add") && /Register host/.test($("#view").textContent), "hosts view");
  $("#add").click();
  await openModal("host form");
  submitModal((el) => { el.name.value = "w2"; el.ip.value = "10.0.0.9"; el.password.value = "pw"; });
  await until(() => rowWith(/w2.*10\.0\.0\.9/), "registered host row", 30000);
  log("host-registered", {row: rowWith(/w2/).textContent.replace(/\s+/g, " ").trim()});
  await runOp("add-worker", (el) => { el.host.value = "w2"; }, "add-worker");
  win.location.hash = "#/cluster/uiflow/nodes";
  const nodeRow = await until(() => rowWith(/10\.0\.0\.9/), "new worker in the nodes tab");
  log("worker-added", {nodes: doc.querySelectorAll("#tab table tr").length - 1, row: nodeRow.textContent.replace(/\s+/g, " ").trim()});

  // ------------------------------------------------------------------ backup storage (settings) -> backup operation
  win.location.hash = "#/settings/backup-storage";
  await until(() => $("#add") && /Backup storage/.test($("#view").textContent), "backup-storage tab");
  $("#add").click();
  await openModal("backup storage form");
  submitModal((el) => { el.name.value = "ui-local"; el.type.value = "LOCAL"; el.credentials.value = JSON.stringify({path: BACKUP_DIR}); });
  await until(() => rowWith(/ui-local/), "backup storage row");
  await runOp("backup", () => {}, "backup");
  win.location.hash = "#/cluster/uiflow/backup";
  await until(() => $("#strat") && doc.querySelectorAll("#tab table tr").length >= 2, "backup listed in the backup tab");
  log("backup-done", {backups: doc.querySelectorAll("#tab table").slice(-1)[0].querySelectorAll("tr").length - 1});

  // ------------------------------------------------------------------ settings (LDAP tab) and a user
  win.location.hash = "#/settings/ldap";
  const sf = await until(() => $("#sf"), "ldap settings form");
  sf.elements.AUTH_LDAP_SERVER_URI.value = "ldap://ldap.example.org:389";
  sf.dispatchEvent(new Event("submit", {bubbles: true}));
  await until(() => $("#sf-msg").textContent === "saved", "ldap settings saved");
  win.location.hash = "#/settings/system";
  await until(() => $("#sf") && $("#sf").elements.ntp_server, "system tab");
  win.location.hash = "#/settings/ldap";
  await until(() => $("#sf") && $("#sf").elements.AUTH_LDAP_SERVER_URI && $("#sf").elements.AUTH_LDAP_SERVER_URI.value === "ldap://ldap.example.org:389", "ldap setting read back");
  win.location.hash = "#/users";
  await until(() => $("#add") && /Users/.test($("#view").textContent), "users view");
  $("#add").click();
  await openModal("user form");
  submitModal((el) => { el.username.value = "alice"; el.email.value = "alice@example.org"; el.password.value = "Secret-123"; });
  await until(() => rowWith(/alice/), "user row");
  log("settings-and-user", {ldap: "ldap://ldap.example.org:389"});

  // ------------------------------------------------------------------ dashboard filters (item -> cluster list)
  win.location.hash = "#/dashboard";
  await until(() => $("#d-item") && /Cluster status/.test($("#view").textContent), "dashboard cards");
  const itemSel = $("#d-item");
  itemSel.value = itemSel.options[1].value;  // the seeded default item
  itemSel.dispatchEvent(new Event("change"));
  await until(() => /^#\/dashboard\/[^/]+\/all$/.test(win.location.hash) && rowWith(/uiflow/), "cluster under its item");
  $("#d-refresh").click();  // no Kubernetes API on the simulated farm: the refresh fails quietly, the view re-renders
  await until(() => $("#d-item") && /Statistics/.test($("#view").textContent), "dashboard after refresh");
  log("dashboard", {cards: doc.querySelectorAll("#view h3").map((h) => h.textContent)});

  // ------------------------------------------------------------------ task monitor (the reference's Flower)
  win.location.hash = "#/tasks";
  await until(() => /Task monitor/.test($("#view").textContent) && /online/.test($("#view").textContent), "task monitor with an online worker");
  const kids = $("#view").children;
  const h = kids.findIndex((el) => el.localName === "h3" && el.textContent === "Recent jobs");
  const jobTable = kids.slice(h + 1).find((el) => el.localName === "table");
  const jobRows = jobTable.querySelectorAll("tr").length - 1;
  log("task-monitor", {recent_jobs: jobRows});
  if (alerts.length) throw new Error("unexpected alerts: " + alerts.join("; "));
  sockets.forEach((s) => s.close());
  log("done");
}

main().then(() => process.exit(0), (e) => { console.log(JSON.stringify({error: String(e && e.stack || e)})); process.exit(1); });
