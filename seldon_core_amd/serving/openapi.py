"""OpenAPI (Swagger 2.0) descriptions of the external engine API and the
internal component API (reference openapi/engine.oas3.json, openapi/wrapper.oas3.json,
served at ``/seldon.json`` by python/seldon_core/wrapper.py:33-35)."""
from __future__ import annotations

import json
from typing import Dict

_MSG = {"$ref": "#/definitions/SeldonMessage"}
_DEFS = {
    "SeldonMessage": {"type": "object", "properties": {
        "status": {"$ref": "#/definitions/Status"}, "meta": {"$ref": "#/definitions/Meta"},
        "data": {"$ref": "#/definitions/DefaultData"}, "binData": {"type": "string", "format": "byte"},
        "strData": {"type": "string"}, "jsonData": {"type": "object"}}},
    "DefaultData": {"type": "object", "properties": {
        "names": {"type": "array", "items": {"type": "string"}},
        "tensor": {"$ref": "#/definitions/Tensor"}, "ndarray": {"type": "array", "items": {}},
        "tftensor": {"type": "object"}}},
    "Tensor": {"type": "object", "properties": {"shape": {"type": "array", "items": {"type": "integer"}},
                                                 "values": {"type": "array", "items": {"type": "number"}}}},
    "Meta": {"type": "object", "properties": {
        "puid": {"type": "string"}, "tags": {"type": "object"},
        "routing": {"type": "object", "additionalProperties": {"type": "integer"}},
        "requestPath": {"type": "object", "additionalProperties": {"type": "string"}},
        "metrics": {"type": "array", "items": {"$ref": "#/definitions/Metric"}}}},
    "Metric": {"type": "object", "properties": {"key": {"type": "string"},
                                                 "type": {"type": "string", "enum": ["COUNTER", "GAUGE", "TIMER"]},
                                                 "value": {"type": "number"}, "tags": {"type": "object"}}},
    "Status": {"type": "object", "properties": {"code": {"type": "integer"}, "info": {"type": "string"},
                                                 "reason": {"type": "string"},
                                                 "status": {"type": "string", "enum": ["SUCCESS", "FAILURE"]}}},
    "SeldonMessageList": {"type": "object", "properties": {"seldonMessages": {"type": "array", "items": _MSG}}},
    "Feedback": {"type": "object", "properties": {"request": _MSG, "response": _MSG, "reward": {"type": "number"},
                                                   "truth": _MSG}},
}


def _op(summary: str, body_ref: str) -> Dict:
    return {"post": {"summary": summary, "consumes": ["application/json"], "produces": ["application/json"],
                     "parameters": [{"in": "body", "name": "body", "required": True,
                                     "schema": {"$ref": f"#/definitions/{body_ref}"}}],
                     "responses": {"200": {"description": "SeldonMessage", "schema": _MSG}}}}


def engine_spec() -> Dict:
    return {"swagger": "2.0", "info": {"title": "Seldon external API (MI355X engine)", "version": "0.1"},
            "paths": {"/api/v0.1/predictions": _op("predict through the inference graph", "SeldonMessage"),
                      "/api/v0.1/feedback": _op("send feedback (reward) along the response's routing", "Feedback")},
            "definitions": _DEFS}


def wrapper_spec() -> Dict:
    paths = {f"/{p}": _op(p, ref) for p, ref in [
        ("predict", "SeldonMessage"), ("transform-input", "SeldonMessage"), ("transform-output", "SeldonMessage"),
        ("route", "SeldonMessage"), ("aggregate", "SeldonMessageList"), ("send-feedback", "Feedback")]}
    return {"swagger": "2.0", "info": {"title": "Seldon internal component API (MI355X engine)", "version": "0.1"},
            "paths": paths, "definitions": _DEFS}


def wrapper_spec_json() -> str:
    return json.dumps(wrapper_spec())
