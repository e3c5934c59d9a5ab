// Runs the web wallet's script (nodexa_chain_core_amd/gui/index.html) under Node.js against a
// live node: a minimal DOM stub stands in for the browser and fetch() goes to the node's JSON-RPC
// port with basic auth. Drives the pages like a user and prints what they show as one JSON line.
//
//   node gui_harness.js <index.html> <rpc port> <user:password> <send-to address>
"use strict";
const fs = require("fs");
const http = require("http");
const vm = require("vm");

const [html, port, auth, dest] = process.argv.slice(2);
const src = fs.readFileSync(html, "utf8");
const script = src.slice(src.indexOf("<script>") + 8, src.lastIndexOf("</script>"));

const elements = {};
function el(id) {
  if (!elements[id]) {
    const cls = new Set();
    elements[id] = {id, textContent: "", innerHTML: "", value: "", checked: false, className: "", dataset: {},
                    scrollTop: 0, scrollHeight: 0, onclick: null, onchange: null, onkeydown: null,
                    classList: {toggle: (c, on) => (on ? cls.add(c) : cls.delete(c)), has: (c) => cls.has(c)}};
  }
  return elements[id];
}
const tabs = [...src.matchAll(/data-tab="(\w+)"/g)].map((m) => m[1]);
const buttons = tabs.map((t) => Object.assign(el("tab-" + t), {dataset: {tab: t}}));
const sections = [...src.matchAll(/<section id="(\w+)"/g)].map((m) => el(m[1]));
const document = {
  getElementById: el,
  querySelectorAll: (sel) => (sel === "#tabs button" ? buttons : sel === "section" ? sections : []),
};
function fetch(path, opts) {
  return new Promise((resolve, reject) => {
    const req = http.request({host: "127.0.0.1", port: Number(port), path, method: opts.method,
                              headers: Object.assign({Authorization: "Basic " + Buffer.from(auth).toString("base64")},
                                                     opts.headers)},
      (res) => {
        let body = "";
        res.on("data", (d) => (body += d));
        res.on("end", () => resolve({json: async () => JSON.parse(body)}));
      });
    req.on("error", reject);
    req.end(opts.body);
  });
}
const ctx = vm.createContext({document, fetch, setInterval: () => 0, console, Promise, JSON, Number, String,
                              Object, Date, Math, Error, Set});
vm.runInContext(script, ctx);
const $ = el;
const tick = () => new Promise((r) => setTimeout(r, 300));

(async () => {
  const out = {};
  await tick();  // the initial refresh() of the overview
  out.available = $("bal-available").textContent;
  out.blocks = $("chain-blocks").textContent;
  out.status = $("status").textContent;
  out.recentRows = ($("recent").innerHTML.match(/<tr>/g) || []).length - 1;
  buttons[tabs.indexOf("receive")].onclick();
  await tick();
  $("recv-label").value = "harness";
  await $("recv-new").onclick();
  out.newAddress = $("recv-result").textContent;
  out.receiveClass = $("recv-result").className;
  $("send-addr").value = dest;
  $("send-amount").value = "2.5";
  $("send-comment").value = "gui harness";
  await $("send-btn").onclick();
  out.send = $("send-result").textContent;
  buttons[tabs.indexOf("transactions")].onclick();
  await tick();
  out.txRows = ($("tx-list").innerHTML.match(/<tr>/g) || []).length - 1;
  buttons[tabs.indexOf("mining")].onclick();
  await tick();
  out.mining = $("mining-info").innerHTML.indexOf("Hash rate") >= 0;
  buttons[tabs.indexOf("peers")].onclick();
  await tick();
  out.peers = $("net-totals").textContent || $("net-totals").innerHTML;
  $("console-in").value = "getblockcount";
  await $("console-in").onkeydown({key: "Enter"});
  $("console-in").value = 'getblockhash 1';
  await $("console-in").onkeydown({key: "Enter"});
  out.console = $("console-out").textContent;
  out.activeSection = sections.filter((s) => s.classList.has("active")).map((s) => s.id);
  console.log(JSON.stringify(out));
})().catch((e) => { console.error(e.stack || e); process.exit(1); });
