// A small DOM for running the web UI (kubeoperator_amd/control/ui/app.js) under plain node 12 in tests: elements
// with attributes / children / events, an HTML parser behind innerHTML, querySelector(All) for the selector
// subset the UI uses (tag, #id, .class, [attr], [attr=value], descendant and comma lists), form controls (value,
// checked, named access form.<name>, FormData), location.hash + hashchange, localStorage. No layout, no CSS.
"use strict";

const VOID = new Set(["input", "br", "img", "hr", "meta", "link", "col", "area", "base", "embed", "source", "track", "wbr"]);
const ENT = {amp: "&", lt: "<", gt: ">", quot: '"', apos: "'", nbsp: " ", mdash: "—", ndash: "–", middot: "·", times: "×", hellip: "…"};
const decode = (s) => s.replace(/&(#x[0-9a-f]+|#\d+|\w+);/gi, (m, e) => {
  if (e[0] === "#") return String.fromCodePoint(e[1] === "x" || e[1] === "X" ? parseInt(e.slice(2), 16) : parseInt(e.slice(1), 10));
  return ENT[e] !== undefined ? ENT[e] : m;
});
const escText = (s) => String(s).replace(/&/g, "&amp;").replace(/</g, "&lt;").replace(/>/g, "&gt;");

class Event {
  constructor(type, opts) { this.type = type; this.bubbles = !!(opts && opts.bubbles); this.defaultPrevented = false; this._stop = false; this.target = null; }
  preventDefault() { this.defaultPrevented = true; }
  stopPropagation() { this._stop = true; }
}

class Node {
  constructor() { this.parentNode = null; this.childNodes = []; this.listeners = {}; }
  addEventListener(type, fn) { (this.listeners[type] = this.listeners[type] || []).push(fn); }
  removeEventListener(type, fn) { this.listeners[type] = (this.listeners[type] || []).filter((f) => f !== fn); }
  dispatchEvent(ev) {
    if (!ev.target) ev.target = this;
    let el = this;
    while (el) {
      ev.currentTarget = el;
      for (const f of (el.listeners[ev.type] || []).slice()) f.call(el, ev);
      const h = el["on" + ev.type];
      if (typeof h === "function") h.call(el, ev);
      if (ev._stop || !ev.bubbles) break;
      el = el.parentNode;
    }
    return !ev.defaultPrevented;
  }
}

class Text extends Node {
  constructor(t) { super(); this.nodeType = 3; this.data = t; }
  get textContent() { return this.data; }
  set textContent(v) { this.data = String(v); }
  get outerHTML() { return escText(this.data); }
}

// forms expose their named controls as properties, ahead of the element's own (HTMLFormElement's
// [LegacyOverrideBuiltIns]): form.name is the control named "name" when there is one
const FORM_HANDLER = {
  get(target, prop, recv) {
    if (typeof prop === "string" && prop[0] !== "_") {
      const named = target._named(prop);
      if (named) return named;
    }
    return Reflect.get(target, prop, recv);
  },
  set(target, prop, value) { target[prop] = value; return true; },
};

class Element extends Node {
  constructor(tag, doc) {
    super();
    this.nodeType = 1;
    this.localName = tag.toLowerCase();
    this.tagName = tag.toUpperCase();
    this.attrs = new Map();
    this.style = {};
    this.ownerDocument = doc;
    this.scrollTop = 0;
    this.scrollHeight = 0;
    this._value = undefined;
    this._checked = undefined;
    this._selected = undefined;
    if (this.localName === "form") return new Proxy(this, FORM_HANDLER);
  }
  getAttribute(n) { return this.attrs.has(n) ? this.attrs.get(n) : null; }
  setAttribute(n, v) { this.attrs.set(n, String(v)); }
  hasAttribute(n) { return this.attrs.has(n); }
  removeAttribute(n) { this.attrs.delete(n); }
  get id() { return this.getAttribute("id") || ""; }
  set id(v) { this.setAttribute("id", v); }
  get name() { return this.getAttribute("name") || ""; }
  get type() { return (this.getAttribute("type") || (this.localName === "button" ? "submit" : "text")).toLowerCase(); }
  get href() { return this.getAttribute("href") || ""; }
  set href(v) { this.setAttribute("href", v); }
  get className() { return this.getAttribute("class") || ""; }
  set className(v) { this.setAttribute("class", v); }
  get classList() {
    const el = this;
    const list = () => el.className.split(/\s+/).filter(Boolean);
    const api = {
      add: (...c) => { const s = list(); c.forEach((x) => { if (!s.includes(x)) s.push(x); }); el.className = s.join(" "); },
      remove: (...c) => { el.className = list().filter((x) => !c.includes(x)).join(" "); },
      contains: (c) => list().includes(c),
      toggle: (c, force) => { const has = list().includes(c); const want = force === undefined ? !has : !!force; if (want) api.add(c); else api.remove(c); return want; },
    };
    return api;
  }
  get dataset() {
    const el = this;
    return new Proxy({}, {
      get(_, k) { const n = "data-" + String(k).replace(/[A-Z]/g, (c) => "-" + c.toLowerCase()); return el.hasAttribute(n) ? el.getAttribute(n) : undefined; },
      set(_, k, v) { el.setAttribute("data-" + String(k).replace(/[A-Z]/g, (c) => "-" + c.toLowerCase()), v); return true; },
    });
  }
  get children() { return this.childNodes.filter((n) => n.nodeType === 1); }
  appendChild(n) { if (n.parentNode) n.parentNode.removeChild(n); n.parentNode = this; this.childNodes.push(n); return n; }
  removeChild(n) { this.childNodes = this.childNodes.filter((c) => c !== n); n.parentNode = null; return n; }
  remove() { if (this.parentNode) this.parentNode.removeChild(this); }
  get textContent() { return this.childNodes.map((c) => c.textContent).join(""); }
  set textContent(v) { this.childNodes = []; if (v !== "" && v !== null && v !== undefined) this.appendChild(new Text(String(v))); }
  get innerText() { return this.textContent; }
  get innerHTML() { return this.childNodes.map((c) => c.outerHTML).join(""); }
  set innerHTML(html) { this.childNodes = []; parseHTML(String(html), this, this.ownerDocument); }
  get outerHTML() {
    const a = [...this.attrs].map(([k, v]) => ` ${k}="${String(v).replace(/"/g, "&quot;")}"`).join("");
    return VOID.has(this.localName) ? `<${this.localName}${a}>` : `<${this.localName}${a}>${this.innerHTML}</${this.localName}>`;
  }
  // ------------------------------------------------------------- form controls
  get options() { return this.querySelectorAll("option"); }
  get value() {
    if (this.localName === "select") {
      const opts = this.options;
      const sel = opts.find((o) => o._selected === true) || opts.find((o) => o._selected === undefined && o.hasAttribute("selected")) || opts[0];
      return sel ? sel.value : "";
    }
    if (this.localName === "option") return this.hasAttribute("value") ? this.getAttribute("value") : this.textContent;
    if (this.localName === "textarea") return this._value !== undefined ? this._value : this.textContent;
    return this._value !== undefined ? this._value : (this.getAttribute("value") || "");
  }
  set value(v) {
    if (this.localName === "select") { this.options.forEach((o) => { o._selected = o.value === String(v); }); return; }
    this._value = String(v);
  }
  get checked() { return this._checked !== undefined ? this._checked : this.hasAttribute("checked"); }
  set checked(v) { this._checked = !!v; }
  get elements() {
    const el = this;
    return new Proxy({}, {get(_, k) { return el._named(String(k)); }});
  }
  _named(n) { return this.querySelectorAll("input, select, textarea, button").find((x) => x.getAttribute("name") === n) || null; }
  click() {
    const ev = new Event("click", {bubbles: true});
    this.dispatchEvent(ev);
    if (ev.defaultPrevented) return;
    if (this.localName === "button" && this.type === "submit") {
      let f = this.parentNode;
      while (f && f.localName !== "form") f = f.parentNode;
      if (f) f.dispatchEvent(new Event("submit", {bubbles: true}));
    }
    if (this.localName === "a" && this.href.startsWith("#") && this.ownerDocument.window) this.ownerDocument.window.location.hash = this.href;
  }
  // ------------------------------------------------------------- selectors
  querySelectorAll(sel) { const out = []; const groups = parseSelector(sel); walk(this, (el) => { if (groups.some((g) => matchComplex(el, g, this))) out.push(el); }); return out; }
  querySelector(sel) { return this.querySelectorAll(sel)[0] || null; }
  matches(sel) { return parseSelector(sel).some((g) => matchComplex(this, g, null)); }
  closest(sel) { let el = this; while (el && el.nodeType === 1) { if (el.matches(sel)) return el; el = el.parentNode; } return null; }
}

function walk(root, fn) {
  for (const c of root.childNodes) {
    if (c.nodeType !== 1) continue;
    fn(c);
    walk(c, fn);
  }
}

// selector = comma list of complex selectors; complex = compounds joined by descendant whitespace
function parseSelector(sel) {
  return sel.split(",").map((g) => g.trim().match(/(?:[^\s"'\[]+|\[[^\]]*\])+/g).map((compound) => {
    const parts = {tag: null, id: null, classes: [], attrs: []};
    const re = /([a-zA-Z][\w-]*)|#([\w-]+)|\.([\w-]+)|\[([\w-]+)(?:=(?:"([^"]*)"|'([^']*)'|([^\]]*)))?\]/g;
    let m;
    while ((m = re.exec(compound))) {
      if (m[1]) parts.tag = m[1].toLowerCase();
      else if (m[2]) parts.id = m[2];
      else if (m[3]) parts.classes.push(m[3]);
      else parts.attrs.push([m[4], m[5] !== undefined ? m[5] : m[6] !== undefined ? m[6] : m[7]]);
    }
    return parts;
  }));
}

function matchCompound(el, p) {
  if (p.tag && el.localName !== p.tag) return false;
  if (p.id && el.id !== p.id) return false;
  for (const c of p.classes) if (!el.classList.contains(c)) return false;
  for (const [a, v] of p.attrs) { if (!el.hasAttribute(a)) return false; if (v !== undefined && el.getAttribute(a) !== v) return false; }
  return true;
}

function matchComplex(el, compounds, scope) {
  if (!matchCompound(el, compounds[compounds.length - 1])) return false;
  let i = compounds.length - 2;
  let anc = el.parentNode;
  while (i >= 0) {
    while (anc && anc.nodeType === 1 && anc !== scope && !matchCompound(anc, compounds[i])) anc = anc.parentNode;
    if (!anc || anc.nodeType !== 1 || anc === scope) return false;
    i--;
    anc = anc.parentNode;
  }
  return true;
}

// ------------------------------------------------------------------ HTML parser (enough for the UI's markup)
function parseHTML(html, parent, doc) {
  const stack = [parent];
  const re = /<!--[\s\S]*?-->|<\/([a-zA-Z][\w-]*)\s*>|<([a-zA-Z][\w-]*)((?:\s+[^\s"'>\/=]+(?:\s*=\s*(?:"[^"]*"|'[^']*'|[^\s>]+))?)*)\s*(\/?)>|([^<]+|<)/g;
  let m;
  while ((m = re.exec(html))) {
    const top = stack[stack.length - 1];
    if (m[0].startsWith("<!--")) continue;
    if (m[1]) {  // end tag: pop to the matching element
      const tag = m[1].toLowerCase();
      for (let i = stack.length - 1; i > 0; i--) if (stack[i].localName === tag) { stack.length = i; break; }
    } else if (m[2]) {
      const el = doc.createElement(m[2]);
      const ar = /([^\s"'>\/=]+)(?:\s*=\s*(?:"([^"]*)"|'([^']*)'|([^\s>]+)))?/g;
      let a;
      while ((a = ar.exec(m[3] || ""))) el.setAttribute(a[1].toLowerCase(), decode(a[2] !== undefined ? a[2] : a[3] !== undefined ? a[3] : a[4] !== undefined ? a[4] : ""));
      top.appendChild(el);
      if (el.localName === "script" || el.localName === "style") {  // raw text up to the end tag
        const end = html.toLowerCase().indexOf(`</${el.localName}`, re.lastIndex);
        const stop = end < 0 ? html.length : end;
        if (stop > re.lastIndex) el.appendChild(new Text(html.slice(re.lastIndex, stop)));
        re.lastIndex = stop;
        continue;
      }
      if (!VOID.has(el.localName) && !m[4]) stack.push(el);
    } else if (m[5]) {
      top.appendChild(new Text(decode(m[5])));
    }
  }
}

class Document extends Node {
  constructor() {
    super();
    this.nodeType = 9;
    this.documentElement = new Element("html", this);
    this.head = this.documentElement.appendChild(new Element("head", this));
    this.body = this.documentElement.appendChild(new Element("body", this));
    this.documentElement.parentNode = this;
    this.childNodes = [this.documentElement];
  }
  createElement(tag) { return new Element(tag, this); }
  createTextNode(t) { return new Text(t); }
  getElementById(id) { return this.documentElement.querySelector("#" + id); }
  querySelector(s) { return this.documentElement.querySelector(s); }
  querySelectorAll(s) { return this.documentElement.querySelectorAll(s); }
}

class FormData {
  constructor(form) {
    this._e = [];
    if (!form) return;
    for (const el of form.querySelectorAll("input, select, textarea")) {
      const n = el.getAttribute("name");
      if (!n || el.hasAttribute("disabled")) continue;
      if (el.localName === "input" && (el.type === "checkbox" || el.type === "radio") && !el.checked) continue;
      if (el.localName === "input" && el.type === "file") continue;
      this._e.push([n, el.localName === "input" && el.type === "checkbox" ? (el.getAttribute("value") || "on") : el.value]);
    }
  }
  append(k, v) { this._e.push([k, v]); }
  get(k) { const e = this._e.find((x) => x[0] === k); return e ? e[1] : null; }
  entries() { return this._e[Symbol.iterator](); }
  [Symbol.iterator]() { return this._e[Symbol.iterator](); }
}

class Storage {
  constructor() { this._m = new Map(); }
  getItem(k) { return this._m.has(k) ? this._m.get(k) : null; }
  setItem(k, v) { this._m.set(k, String(v)); }
  removeItem(k) { this._m.delete(k); }
}

function makeWindow(host) {
  const document = new Document();
  const win = new Node();
  document.window = win;
  let hash = "";
  win.location = {
    protocol: "http:", host,
    get hash() { return hash; },
    set hash(v) { const nv = v.startsWith("#") ? v : "#" + v; if (nv !== hash) { hash = nv; setImmediate(() => win.dispatchEvent(new Event("hashchange"))); } },
  };
  win.document = document;
  win.localStorage = new Storage();
  win.Event = Event;
  win.FormData = FormData;
  return win;
}

module.exports = {Document, Element, Event, FormData, Storage, makeWindow, parseHTML};
