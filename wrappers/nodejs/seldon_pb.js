"use strict";
// Dependency-free protobuf codec for the Seldon prediction API
// (proto/prediction.proto, package seldon.protos): SeldonMessage,
// SeldonMessageList and Feedback, converted to / from the same plain-object
// shape the REST API uses ({data: {names, tensor: {shape, values}} | {ndarray}},
// meta, status, binData (base64), strData, jsonData).  The reference NodeJS
// wrapper uses the generated google-protobuf classes
// (wrappers/s2i/nodejs/prediction_pb.js); this image has no npm registry, so
// the wire format is written by hand -- only what the API carries.

// ---------------------------------------------------------------- writer
class Writer {
  constructor() {
    this.parts = [];
    this.len = 0;
  }
  push(buf) {
    this.parts.push(buf);
    this.len += buf.length;
  }
  varint(v) {
    const out = [];
    if (v < 0) {  // int32 negatives are 10-byte two's complement varints
      let lo = v >>> 0, hi = 0xffffffff;
      for (let i = 0; i < 9; i++) {
        out.push((lo & 0x7f) | 0x80);
        lo = (lo >>> 7) | ((hi & 0x7f) << 25);
        hi >>>= 7;
      }
      out.push(1);
    } else {
      while (v > 0x7f) {
        out.push((v & 0x7f) | 0x80);
        v = Math.floor(v / 128);
      }
      out.push(v);
    }
    this.push(Buffer.from(out));
  }
  tag(field, wire) { this.varint(field * 8 + wire); }
  bytes(field, buf) {
    this.tag(field, 2);
    this.varint(buf.length);
    this.push(buf);
  }
  string(field, s) { this.bytes(field, Buffer.from(String(s), "utf8")); }
  message(field, w) { this.bytes(field, w.finish()); }
  double(field, v) {
    this.tag(field, 1);
    const b = Buffer.alloc(8);
    b.writeDoubleLE(v, 0);
    this.push(b);
  }
  float(field, v) {
    this.tag(field, 5);
    const b = Buffer.alloc(4);
    b.writeFloatLE(v, 0);
    this.push(b);
  }
  int(field, v) {
    this.tag(field, 0);
    this.varint(v | 0);
  }
  finish() { return Buffer.concat(this.parts, this.len); }
}

// ---------------------------------------------------------------- reader
class Reader {
  constructor(buf) {
    this.buf = buf;
    this.pos = 0;
  }
  eof() { return this.pos >= this.buf.length; }
  varint() {
    let result = 0, mul = 1, b;
    do {
      if (this.pos >= this.buf.length) throw new Error("truncated varint");
      b = this.buf[this.pos++];
      result += (b & 0x7f) * mul;
      mul *= 128;
    } while (b & 0x80);
    return result;
  }
  int32() {  // low 32 bits of the varint (negatives are 10-byte two's complement)
    let lo = 0, shift = 0, b;
    do {
      if (this.pos >= this.buf.length) throw new Error("truncated varint");
      b = this.buf[this.pos++];
      if (shift < 32) lo |= (b & 0x7f) << shift;
      shift += 7;
    } while (b & 0x80);
    return lo | 0;
  }
  bytes() {
    const n = this.varint();
    if (this.pos + n > this.buf.length) throw new Error("truncated field");
    const b = this.buf.subarray(this.pos, this.pos + n);
    this.pos += n;
    return b;
  }
  double() {
    const v = this.buf.readDoubleLE(this.pos);
    this.pos += 8;
    return v;
  }
  float() {
    const v = this.buf.readFloatLE(this.pos);
    this.pos += 4;
    return v;
  }
  skip(wire) {
    if (wire === 0) this.varint();
    else if (wire === 1) this.pos += 8;
    else if (wire === 2) this.bytes();
    else if (wire === 5) this.pos += 4;
    else throw new Error("unsupported wire type " + wire);
  }
  // iterate fields: fn(field, wire) must consume the value
  each(fn) {
    while (!this.eof()) {
      const t = this.varint();
      fn(Math.floor(t / 8), t & 7);
    }
  }
}

// --------------------------------------------- google.protobuf.Value / ListValue / Struct
function encodeValue(v) {
  const w = new Writer();
  if (v === null || v === undefined) w.int(1, 0);
  else if (typeof v === "number") w.double(2, v);
  else if (typeof v === "string") w.string(3, v);
  else if (typeof v === "boolean") w.int(4, v ? 1 : 0);
  else if (Array.isArray(v)) w.message(6, encodeList(v));
  else if (typeof v === "object") w.message(5, encodeStruct(v));
  else w.string(3, String(v));
  return w;
}
function encodeList(arr) {
  const w = new Writer();
  for (const x of arr) w.message(1, encodeValue(x));
  return w;
}
function encodeStruct(obj) {
  const w = new Writer();
  for (const k of Object.keys(obj)) {
    const e = new Writer();
    e.string(1, k);
    e.message(2, encodeValue(obj[k]));
    w.message(1, e);
  }
  return w;
}
function decodeValue(buf) {
  const r = new Reader(buf);
  let v = null;
  r.each((f, wire) => {
    if (f === 1) { r.varint(); v = null; }
    else if (f === 2) v = r.double();
    else if (f === 3) v = r.bytes().toString("utf8");
    else if (f === 4) v = r.varint() !== 0;
    else if (f === 5) v = decodeStruct(r.bytes());
    else if (f === 6) v = decodeList(r.bytes());
    else r.skip(wire);
  });
  return v;
}
function decodeList(buf) {
  const r = new Reader(buf), out = [];
  r.each((f, wire) => (f === 1 ? out.push(decodeValue(r.bytes())) : r.skip(wire)));
  return out;
}
function decodeMapEntry(buf, decodeVal) {
  const r = new Reader(buf);
  let k = "", v = decodeVal(null);
  r.each((f, wire) => {
    if (f === 1) k = r.bytes().toString("utf8");
    else if (f === 2) v = decodeVal(r, wire);
    else r.skip(wire);
  });
  return [k, v];
}
function decodeStruct(buf) {
  const r = new Reader(buf), out = {};
  r.each((f, wire) => {
    if (f !== 1) return r.skip(wire);
    const [k, v] = decodeMapEntry(r.bytes(), (rr) => (rr ? decodeValue(rr.bytes()) : null));
    out[k] = v;
  });
  return out;
}

// ------------------------------------------------------------ Seldon messages
const METRIC_TYPES = ["COUNTER", "GAUGE", "TIMER"];

function encodeMeta(m) {
  const w = new Writer();
  if (m.puid) w.string(1, m.puid);
  for (const [k, v] of Object.entries(m.tags || {})) {
    const e = new Writer();
    e.string(1, k);
    e.message(2, encodeValue(v));
    w.message(2, e);
  }
  for (const [k, v] of Object.entries(m.routing || {})) {
    const e = new Writer();
    e.string(1, k);
    e.int(2, v);
    w.message(3, e);
  }
  for (const [k, v] of Object.entries(m.requestPath || {})) {
    const e = new Writer();
    e.string(1, k);
    e.string(2, v);
    w.message(4, e);
  }
  for (const mt of m.metrics || []) {
    const e = new Writer();
    e.string(1, mt.key || "");
    const t = METRIC_TYPES.indexOf(mt.type || "COUNTER");
    if (t > 0) e.int(2, t);
    e.float(3, Number(mt.value || 0));
    for (const [k, v] of Object.entries(mt.tags || {})) {
      const te = new Writer();
      te.string(1, k);
      te.string(2, String(v));
      e.message(4, te);
    }
    w.message(5, e);
  }
  return w;
}
function decodeMeta(buf) {
  const r = new Reader(buf), m = {};
  r.each((f, wire) => {
    if (f === 1) m.puid = r.bytes().toString("utf8");
    else if (f === 2) {
      const [k, v] = decodeMapEntry(r.bytes(), (rr) => (rr ? decodeValue(rr.bytes()) : null));
      (m.tags = m.tags || {})[k] = v;
    } else if (f === 3) {
      const [k, v] = decodeMapEntry(r.bytes(), (rr) => (rr ? rr.int32() : 0));
      (m.routing = m.routing || {})[k] = v;
    } else if (f === 4) {
      const [k, v] = decodeMapEntry(r.bytes(), (rr) => (rr ? rr.bytes().toString("utf8") : ""));
      (m.requestPath = m.requestPath || {})[k] = v;
    } else if (f === 5) {
      const mr = new Reader(r.bytes()), mt = { key: "", type: "COUNTER", value: 0 };
      mr.each((g, wg) => {
        if (g === 1) mt.key = mr.bytes().toString("utf8");
        else if (g === 2) mt.type = METRIC_TYPES[mr.varint()] || "COUNTER";
        else if (g === 3) mt.value = mr.float();
        else if (g === 4) {
          const [k, v] = decodeMapEntry(mr.bytes(), (rr) => (rr ? rr.bytes().toString("utf8") : ""));
          (mt.tags = mt.tags || {})[k] = v;
        } else mr.skip(wg);
      });
      (m.metrics = m.metrics || []).push(mt);
    } else r.skip(wire);
  });
  return m;
}

function encodeStatus(s) {
  const w = new Writer();
  if (s.code) w.int(1, s.code);
  if (s.info) w.string(2, s.info);
  if (s.reason) w.string(3, s.reason);
  if (s.status === "FAILURE") w.int(4, 1);
  return w;
}
function decodeStatus(buf) {
  const r = new Reader(buf), s = { code: 0, info: "", reason: "", status: "SUCCESS" };
  r.each((f, wire) => {
    if (f === 1) s.code = r.int32();
    else if (f === 2) s.info = r.bytes().toString("utf8");
    else if (f === 3) s.reason = r.bytes().toString("utf8");
    else if (f === 4) s.status = r.varint() === 1 ? "FAILURE" : "SUCCESS";
    else r.skip(wire);
  });
  return s;
}

function encodeData(d) {
  const w = new Writer();
  for (const n of d.names || []) w.string(1, n);
  if (d.tensor) {
    const t = new Writer();
    const shape = d.tensor.shape || [];
    if (shape.length) {
      const sw = new Writer();
      for (const x of shape) sw.varint(x | 0);
      t.bytes(1, sw.finish());
    }
    const vals = d.tensor.values || [];
    if (vals.length) {
      const b = Buffer.alloc(8 * vals.length);
      vals.forEach((x, i) => b.writeDoubleLE(Number(x), 8 * i));
      t.bytes(2, b);
    }
    w.message(2, t);
  } else if (d.ndarray !== undefined) {
    w.message(3, encodeList(d.ndarray));
  } else if (d._tftensor) {
    w.bytes(4, d._tftensor);
  }
  return w;
}
function decodeData(buf) {
  const r = new Reader(buf), d = { names: [] };
  r.each((f, wire) => {
    if (f === 1) d.names.push(r.bytes().toString("utf8"));
    else if (f === 2) {
      const tr = new Reader(r.bytes()), t = { shape: [], values: [] };
      tr.each((g, wg) => {
        if (g === 1 && wg === 2) {
          const pr = new Reader(tr.bytes());
          while (!pr.eof()) t.shape.push(pr.int32());
        } else if (g === 1) t.shape.push(tr.int32());
        else if (g === 2 && wg === 2) {
          const b = tr.bytes();
          for (let i = 0; i + 8 <= b.length; i += 8) t.values.push(b.readDoubleLE(i));
        } else if (g === 2) t.values.push(tr.double());
        else tr.skip(wg);
      });
      d.tensor = t;
    } else if (f === 3) d.ndarray = decodeList(r.bytes());
    else if (f === 4) d._tftensor = Buffer.from(r.bytes());
    else r.skip(wire);
  });
  return d;
}

function encodeMessage(m) {
  const w = new Writer();
  if (m.status) w.message(1, encodeStatus(m.status));
  if (m.meta) w.message(2, encodeMeta(m.meta));
  if (m.data) w.message(3, encodeData(m.data));
  else if (m.binData !== undefined) w.bytes(4, Buffer.from(m.binData, "base64"));
  else if (m.strData !== undefined) w.string(5, m.strData);
  else if (m.jsonData !== undefined) w.message(6, encodeValue(m.jsonData));
  return w;
}
function decodeMessage(buf) {
  const r = new Reader(buf), m = {};
  r.each((f, wire) => {
    if (f === 1) m.status = decodeStatus(r.bytes());
    else if (f === 2) m.meta = decodeMeta(r.bytes());
    else if (f === 3) m.data = decodeData(r.bytes());
    else if (f === 4) m.binData = Buffer.from(r.bytes()).toString("base64");
    else if (f === 5) m.strData = r.bytes().toString("utf8");
    else if (f === 6) m.jsonData = decodeValue(r.bytes());
    else r.skip(wire);
  });
  return m;
}

function decodeMessageList(buf) {
  const r = new Reader(buf), out = [];
  r.each((f, wire) => (f === 1 ? out.push(decodeMessage(r.bytes())) : r.skip(wire)));
  return { seldonMessages: out };
}
function encodeMessageList(l) {
  const w = new Writer();
  for (const m of l.seldonMessages || []) w.message(1, encodeMessage(m));
  return w.finish();
}

function decodeFeedback(buf) {
  const r = new Reader(buf), fb = {};
  r.each((f, wire) => {
    if (f === 1) fb.request = decodeMessage(r.bytes());
    else if (f === 2) fb.response = decodeMessage(r.bytes());
    else if (f === 3) fb.reward = r.float();
    else if (f === 4) fb.truth = decodeMessage(r.bytes());
    else r.skip(wire);
  });
  return fb;
}
function encodeFeedback(fb) {
  const w = new Writer();
  if (fb.request) w.message(1, encodeMessage(fb.request));
  if (fb.response) w.message(2, encodeMessage(fb.response));
  if (fb.reward !== undefined) w.float(3, Number(fb.reward));
  if (fb.truth) w.message(4, encodeMessage(fb.truth));
  return w.finish();
}

module.exports = {
  encodeMessage: (m) => encodeMessage(m).finish(),
  decodeMessage,
  encodeMessageList,
  decodeMessageList,
  encodeFeedback,
  decodeFeedback,
  encodeValue: (v) => encodeValue(v).finish(),
  decodeValue,
};
