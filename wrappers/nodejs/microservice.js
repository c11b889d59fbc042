#!/usr/bin/env node
"use strict";
// Seldon microservice wrapper for NodeJS components (SURVEY P1; reference
// wrappers/s2i/nodejs/microservice.js:1-147, model_microservice.js,
// transformer_microservice.js).  Serves a user class over the internal API
// the engine calls for remote graph nodes (csrc/server/remote_unit.cc):
//
//   REST  POST/GET /predict /transform-input /transform-output /route
//         /aggregate /send-feedback  (form field `json=`, a `json` query
//         parameter, or a raw JSON body), GET /health/ping /health/status
//         /ready /live
//   gRPC  /seldon.protos.{Generic,Model,Router,Transformer,OutputTransformer,
//         Combiner,Seldon}/{Predict,TransformInput,TransformOutput,Route,
//         Aggregate,SendFeedback} over HTTP/2 (node's built-in http2)
//
// No npm dependencies (the reference needs express, numjs, grpc): payloads are
// plain nested arrays, the protobuf codec is seldon_pb.js.
//
// User component (a CommonJS module exporting a class, like the reference's
// `--model` file): optional `async init()`, and any of
//   predict(X, names, meta)             -> array
//   transform_input(X, names, meta)     -> array   (identity when absent)
//   transform_output(X, names, meta)    -> array   (identity when absent)
//   route(X, names)                     -> int     (-1 = all children)
//   aggregate(Xs, names_list)           -> array
//   send_feedback(X, names, reward, truth, routing) -> anything
//   tags() -> {}, metrics() -> [{type, key, value}], class_names -> [..]
// Methods may return promises.  Constructor parameters come from
// PREDICTIVE_UNIT_PARAMETERS (JSON [{name, value, type}]), as in the Python
// wrapper (python/seldon_core/microservice.py:parse_parameters).

const http = require("http");
const http2 = require("http2");
const path = require("path");
const querystring = require("querystring");
const url = require("url");
const pb = require("./seldon_pb");

// ------------------------------------------------------------------ args
function parseArgs(argv) {
  const a = { model: "", api: "REST", service: "MODEL", persistence: 0, port: 0, host: "0.0.0.0" };
  const pos = [];
  for (let i = 2; i < argv.length; i++) {
    const t = argv[i];
    if (t.startsWith("--")) {
      const [k, v] = t.includes("=") ? t.slice(2).split(/=(.*)/) : [t.slice(2), argv[++i]];
      a[k] = v;
    } else pos.push(t);
  }
  if (!a.model && pos.length) a.model = pos[0];
  if (!a.api && pos.length > 1) a.api = pos[1];
  a.api = String(a.api).toUpperCase();
  a.service = String(a.service).toUpperCase();
  a.persistence = Number(a.persistence || 0);
  a.port = Number(a.port || process.env.PREDICTIVE_UNIT_SERVICE_PORT || 5000);
  return a;
}

function parseParameters() {
  const raw = process.env.PREDICTIVE_UNIT_PARAMETERS;
  if (!raw) return {};
  const out = {};
  for (const p of JSON.parse(raw)) {
    const t = String(p.type || "STRING").toUpperCase();
    let v = p.value;
    if (t === "INT") v = parseInt(v, 10);
    else if (t === "FLOAT" || t === "DOUBLE") v = parseFloat(v);
    else if (t === "BOOL") v = String(v).toLowerCase() === "true" || v === true;
    out[p.name] = v;
  }
  return out;
}

// The module: an absolute path, or relative to the working directory (the s2i
// source root), or under ./model/ as in the reference wrapper.
function resolveModel(spec) {
  const fs = require("fs");
  const cands = path.isAbsolute(spec) ? [spec] : [path.resolve(spec), path.resolve("model", spec)];
  for (const c of cands)
    for (const f of [c, c + ".js"])
      if (fs.existsSync(f) && fs.statSync(f).isFile()) return f;
  throw new Error("model module " + spec + " not found (tried " + cands.join(", ") + ")");
}

async function loadModel(spec) {
  const M = require(resolveModel(spec));
  const Cls = typeof M === "function" ? M : M.default || M.Model;
  const m = typeof Cls === "function" ? new Cls(parseParameters()) : M;
  if (typeof m.init === "function") await m.init();
  return m;
}

// ------------------------------------------------------------- payloads
class ApiError extends Error {
  constructor(msg, code = 400, reason = "MICROSERVICE_BAD_DATA") {
    super(msg);
    this.code = code;
    this.reason = reason;
  }
}

function reshape(values, shape) {
  if (!shape || shape.length <= 1) return values.slice();
  const [n, ...rest] = shape;
  const step = rest.reduce((a, b) => a * b, 1);
  const out = [];
  for (let i = 0; i < n; i++) out.push(reshape(values.slice(i * step, (i + 1) * step), rest));
  return out;
}

function shapeOf(a) {
  const s = [];
  while (Array.isArray(a)) {
    s.push(a.length);
    a = a[0];
  }
  return s;
}

function flatten(a, out = []) {
  if (Array.isArray(a)) for (const x of a) flatten(x, out);
  else out.push(a);
  return out;
}

// features of a SeldonMessage: nested array (tensor / ndarray), bytes, string or JSON
function features(msg) {
  if (msg.data) {
    const d = msg.data;
    if (d.tensor) return reshape((d.tensor.values || []).map(Number), d.tensor.shape || []);
    if (d.ndarray !== undefined) return d.ndarray;
    if (d.tftensor) throw new ApiError("tftensor payloads are not supported by the NodeJS wrapper");
    return [];
  }
  if (msg.binData !== undefined) return Buffer.from(msg.binData, "base64");
  if (msg.strData !== undefined) return msg.strData;
  if (msg.jsonData !== undefined) return msg.jsonData;
  throw new ApiError("request has no data, binData, strData or jsonData");
}

function classNames(user, arr) {
  if (Array.isArray(user.class_names)) return user.class_names;
  const s = shapeOf(arr);
  const n = s.length > 1 ? s[1] : 0;
  return Array.from({ length: n }, (_, i) => "t:" + i);
}

async function userMeta(user) {
  const meta = {};
  if (typeof user.tags === "function") {
    const t = await user.tags();
    if (t && Object.keys(t).length) meta.tags = t;
  }
  if (typeof user.metrics === "function") {
    const m = await user.metrics();
    if (m && m.length) {
      for (const x of m) {
        if (!x || !["COUNTER", "GAUGE", "TIMER"].includes(x.type) || typeof x.key !== "string" || isNaN(Number(x.value)))
          throw new ApiError("bad metric " + JSON.stringify(x), 500, "MICROSERVICE_BAD_METRIC");
      }
      meta.metrics = m;
    }
  }
  return meta;
}

// response SeldonMessage for `result`, in the request's data encoding
async function respond(user, request, result, names) {
  const out = {};
  if (Buffer.isBuffer(result)) out.binData = result.toString("base64");
  else if (typeof result === "string") out.strData = result;
  else if (Array.isArray(result) || typeof result === "number") {
    const arr = typeof result === "number" ? [result] : result;
    const d = { names: names || classNames(user, arr) };
    if (request.data && request.data.tensor) d.tensor = { shape: shapeOf(arr), values: flatten(arr).map(Number) };
    else d.ndarray = arr;
    out.data = d;
  } else out.jsonData = result;
  const meta = await userMeta(user);
  const reqMeta = request.meta || {};
  if (reqMeta.puid) meta.puid = reqMeta.puid;
  if (Object.keys(meta).length) out.meta = meta;
  return out;
}

function names(msg) {
  return (msg.data && msg.data.names) || [];
}

// --------------------------------------------------------------- methods
const METHODS = {
  async predict(user, req) {
    if (typeof user.predict_raw === "function") return user.predict_raw(req);
    if (typeof user.predict !== "function") throw new ApiError("predict is not implemented", 400, "MICROSERVICE_BAD_METHOD");
    return respond(user, req, await user.predict(features(req), names(req), req.meta || {}));
  },
  async transform_input(user, req) {
    if (typeof user.transform_input_raw === "function") return user.transform_input_raw(req);
    if (typeof user.transform_input !== "function") return req;
    return respond(user, req, await user.transform_input(features(req), names(req), req.meta || {}), undefined);
  },
  async transform_output(user, req) {
    if (typeof user.transform_output_raw === "function") return user.transform_output_raw(req);
    if (typeof user.transform_output !== "function") return req;
    return respond(user, req, await user.transform_output(features(req), names(req), req.meta || {}), undefined);
  },
  async route(user, req) {
    if (typeof user.route_raw === "function") return user.route_raw(req);
    if (typeof user.route !== "function") throw new ApiError("route is not implemented", 400, "MICROSERVICE_BAD_METHOD");
    const r = await user.route(features(req), names(req));
    if (!Number.isInteger(Number(r))) throw new ApiError("route must return an integer", 500, "MICROSERVICE_BAD_ROUTING");
    const out = await respond(user, req, [[Number(r)]], []);
    return out;
  },
  async aggregate(user, list) {
    if (typeof user.aggregate_raw === "function") return user.aggregate_raw(list);
    if (typeof user.aggregate !== "function") throw new ApiError("aggregate is not implemented", 400, "MICROSERVICE_BAD_METHOD");
    const msgs = list.seldonMessages || [];
    if (!msgs.length) throw new ApiError("aggregate needs seldonMessages");
    const res = await user.aggregate(msgs.map(features), msgs.map(names));
    return respond(user, msgs[0], res);
  },
  async send_feedback(user, fb) {
    if (typeof user.send_feedback_raw === "function") return user.send_feedback_raw(fb);
    if (typeof user.send_feedback !== "function") return {};
    const req = fb.request || {};
    const routing = (req.meta && req.meta.routing) || {};
    const truth = fb.truth ? features(fb.truth) : null;
    const r = await user.send_feedback(features(req), names(req), fb.reward || 0, truth, routing);
    return Array.isArray(r) ? respond(user, req, r) : {};
  },
};

function failure(e) {
  const code = e instanceof ApiError ? e.code : 500;
  return {
    code,
    body: { status: { code: -1, info: String(e.message || e), reason: e.reason || "MICROSERVICE_INTERNAL_ERROR", status: "FAILURE" } },
  };
}

// ------------------------------------------------------------------ REST
const REST_ROUTES = {
  "/predict": "predict",
  "/api/v0.1/predictions": "predict",
  "/transform-input": "transform_input",
  "/transform-output": "transform_output",
  "/route": "route",
  "/aggregate": "aggregate",
  "/send-feedback": "send_feedback",
};

function restBody(req, raw) {
  const q = url.parse(req.url, true).query;
  let text = q.json;
  if (!text && raw.length) {
    const ct = String(req.headers["content-type"] || "");
    if (ct.includes("application/x-www-form-urlencoded")) text = querystring.parse(raw.toString("utf8")).json;
    else text = raw.toString("utf8");
  }
  if (!text) throw new ApiError("empty request: expected a json body or a json form field");
  try {
    return JSON.parse(text);
  } catch (e) {
    throw new ApiError("invalid JSON: " + e.message);
  }
}

function serveRest(user, args) {
  let ready = true;
  const server = http.createServer((req, res) => {
    const chunks = [];
    req.on("data", (c) => chunks.push(c));
    req.on("end", async () => {
      const p = url.parse(req.url).pathname;
      const send = (code, obj, type = "application/json") => {
        const body = typeof obj === "string" ? obj : JSON.stringify(obj);
        res.writeHead(code, { "Content-Type": type, "Content-Length": Buffer.byteLength(body) });
        res.end(body);
      };
      try {
        if (p === "/health/ping" || p === "/ping") return send(200, "pong", "text/plain");
        if (p === "/live") return send(200, "live", "text/plain");
        if (p === "/ready") return send(ready ? 200 : 503, ready ? "ready" : "not ready", "text/plain");
        if (p === "/health/status") {
          if (typeof user.health_status === "function") return send(200, await respond(user, {}, await user.health_status()));
          return send(200, { status: { code: 200, status: "SUCCESS" } });
        }
        const method = REST_ROUTES[p];
        if (!method) return send(404, { status: { code: 404, info: "no such endpoint " + p, status: "FAILURE" } });
        const body = restBody(req, Buffer.concat(chunks));
        send(200, await METHODS[method](user, body));
      } catch (e) {
        const f = failure(e);
        send(f.code, f.body);
      }
    });
  });
  server.keepAliveTimeout = 60000;
  server.listen(args.port, args.host, () => console.log(`NodeJS REST microservice (${args.service}) on :${args.port}`));
  return { server, setReady: (r) => (ready = r) };
}

// ------------------------------------------------------------------ gRPC
const GRPC_METHODS = {
  Predict: ["predict", pb.decodeMessage],
  TransformInput: ["transform_input", pb.decodeMessage],
  TransformOutput: ["transform_output", pb.decodeMessage],
  Route: ["route", pb.decodeMessage],
  Aggregate: ["aggregate", pb.decodeMessageList],
  SendFeedback: ["send_feedback", pb.decodeFeedback],
};
const GRPC_SERVICES = new Set(["Generic", "Model", "Router", "Transformer", "OutputTransformer", "Combiner", "Seldon"]);

function frame(buf) {
  const h = Buffer.alloc(5);
  h.writeUInt32BE(buf.length, 1);
  return Buffer.concat([h, buf]);
}

function serveGrpc(user, args) {
  const server = http2.createServer();
  server.on("stream", (stream, headers) => {
    const m = /^\/seldon\.protos\.(\w+)\/(\w+)$/.exec(headers[":path"] || "");
    const chunks = [];
    stream.on("data", (c) => chunks.push(c));
    stream.on("end", async () => {
      let status = 0, message = "", reply = Buffer.alloc(0);
      try {
        if (!m || !GRPC_SERVICES.has(m[1]) || !GRPC_METHODS[m[2]]) {
          status = 12;  // UNIMPLEMENTED
          message = "unknown method " + headers[":path"];
        } else {
          const body = Buffer.concat(chunks);
          if (body.length < 5) throw new ApiError("empty gRPC message");
          if (body[0] !== 0) throw new ApiError("compressed gRPC messages are not supported");
          const n = body.readUInt32BE(1);
          const [name, decode] = GRPC_METHODS[m[2]];
          const out = await METHODS[name](user, decode(body.subarray(5, 5 + n)));
          reply = frame(pb.encodeMessage(out));
        }
      } catch (e) {
        status = e instanceof ApiError ? 3 : 2;  // INVALID_ARGUMENT / UNKNOWN
        message = String(e.message || e);
      }
      if (stream.destroyed) return;
      stream.respond({ ":status": 200, "content-type": "application/grpc" }, { waitForTrailers: true });
      stream.on("wantTrailers", () =>
        stream.sendTrailers({ "grpc-status": String(status), "grpc-message": encodeURIComponent(message) }));
      stream.end(reply);
    });
  });
  server.listen(args.port, args.host, () => console.log(`NodeJS gRPC microservice (${args.service}) on :${args.port}`));
  return { server };
}

// ------------------------------------------------------------------ main
async function main() {
  const args = parseArgs(process.argv);
  if (!args.model) {
    console.error("usage: microservice.js --model <module.js> [--api REST|GRPC] [--service MODEL|...] [--port N]");
    process.exit(2);
  }
  const user = await loadModel(args.model);
  const srv = args.api === "GRPC" ? serveGrpc(user, args) : serveRest(user, args);
  const stop = (sig) => {
    console.log(`${sig}: draining`);
    if (srv.setReady) srv.setReady(false);
    srv.server.close(() => process.exit(0));
    setTimeout(() => process.exit(0), 5000).unref();
  };
  process.on("SIGTERM", () => stop("SIGTERM"));
  process.on("SIGINT", () => stop("SIGINT"));
}

if (require.main === module) {
  main().catch((e) => {
    console.error("failed to start:", e);
    process.exit(1);
  });
}

module.exports = { METHODS, features, respond, reshape };
