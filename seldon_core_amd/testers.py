"""Contract-driven testers.

* ``python -m seldon_core_amd.testers micro <contract.json> <host> <port> ...``
  -- microservice tester (reference python/seldon_core/microservice_tester.py):
  random feature batches generated from a data contract, sent to a
  component's internal API (/predict, /send-feedback) over REST or gRPC.
* ``python -m seldon_core_amd.testers api <contract.json> <host> <port> [deployment] ...``
  -- external API tester (reference api_tester.py) through the engine /
  gateway paths, with optional OAuth.
* :func:`create_seldon_api_testing_file` -- build a contract from a pandas
  DataFrame (reference serving_test_gen.py).

Contract format: ``{"features": [{"name", "ftype": "continuous"|"categorical",
"dtype": "FLOAT"|"INT", "range": [lo, hi] ("inf" allowed), "shape": [...],
"values": [...], "repeat": n}], "targets": [...]}``.
"""
from __future__ import annotations

import argparse
import json
import logging
import sys
from typing import Dict, List, Sequence, Tuple, Union

import numpy as np

from .client import SeldonClient


class SeldonTesterException(Exception):
    pass


def gen_continuous(f_range: Tuple[Union[float, str], Union[float, str]], n) -> np.ndarray:
    lo, hi = f_range
    if lo == "inf" and hi == "inf":
        return np.random.normal(size=n)
    if lo == "inf":
        return hi - np.random.lognormal(size=n)
    if hi == "inf":
        return lo + np.random.lognormal(size=n)
    return np.random.uniform(lo, hi, size=n)


def reconciliate_cont_type(feature: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "FLOAT":
        return feature
    if dtype in ("INT", "INTEGER"):
        return (feature + 0.5).astype(int).astype(float)
    raise SeldonTesterException(f"Unknown dtype in reconciliate_cont_type {dtype}")


def gen_categorical(values: Sequence[str], n) -> np.ndarray:
    return np.array(values)[np.random.randint(len(values), size=n)]


def generate_batch(contract: Dict, n: int, field: str = "features") -> np.ndarray:
    """n random rows for the contract's ``field`` (features or targets)."""
    parts, kinds = [], set()
    for f in contract[field]:
        kinds.add(f["ftype"])
        if f["ftype"] == "continuous":
            shape = [n] + list(f.get("shape", [1]))
            b = np.around(gen_continuous(f.get("range", ["inf", "inf"]), shape), decimals=3)
            b = reconciliate_cont_type(b, f.get("dtype", "FLOAT"))
        elif f["ftype"] == "categorical":
            b = gen_categorical(f["values"], [n, 1])
        else:
            raise SeldonTesterException(f"Unknown feature type {f['ftype']}")
        parts.append(b.reshape(n, -1))
    if len(kinds) == 1:
        return np.concatenate(parts, axis=1)
    return np.concatenate([p.astype(object) for p in parts], axis=1)


def unfold_contract(contract: Dict) -> Dict:
    """Expand ``repeat`` entries (features: name1..nameN; targets: name:0..name:N-1)."""
    out: Dict[str, List[Dict]] = {"features": [], "targets": []}
    for field, fmt in (("features", "{}{}"), ("targets", "{}:{}")):
        for f in contract.get(field, []):
            rep = f.get("repeat")
            if rep is None:
                out[field].append(f)
                continue
            for i in range(rep):
                g = {k: v for k, v in f.items() if k != "repeat"}
                g["name"] = fmt.format(f["name"], i + 1 if field == "features" else i)
                out[field].append(g)
    return out


def feature_names(contract: Dict) -> List[str]:
    return [f["name"] for f in contract["features"]]


def _load(path: str) -> Dict:
    with open(path) as f:
        return unfold_contract(json.load(f))


def run_microservice(args) -> List:
    contract = _load(args.contract)
    sc = SeldonClient(microservice_endpoint=f"{args.host}:{args.port}")
    transport = "grpc" if args.grpc else "rest"
    payload = "tensor" if args.tensor else "ndarray"
    out = []
    for _ in range(args.n_requests):
        batch = generate_batch(contract, args.batch_size)
        if args.prnt:
            print(f"{'-' * 40}\nSENDING NEW REQUEST:\n{batch}")
        r = sc.microservice(data=batch, transport=transport, method="predict", payload_type=payload,
                            names=feature_names(contract))
        if args.endpoint == "send-feedback":
            r = sc.microservice_feedback(prediction_request=r.request, prediction_response=r.response, reward=1.0,
                                         transport=transport)
        if args.prnt:
            print(f"RECEIVED RESPONSE:\n{r.response}\n")
        out.append(r)
    return out


def run_api(args) -> List:
    contract = _load(args.contract)
    endpoint = f"{args.host}:{args.port}"
    gateway = "seldon" if args.oauth_key else "ambassador"
    kw = dict(deployment_name=args.deployment, namespace=args.namespace, gateway=gateway,
              transport="grpc" if args.grpc else "rest", payload_type="tensor" if args.tensor else "ndarray")
    if gateway == "seldon":
        kw.update(oauth_key=args.oauth_key, oauth_secret=args.oauth_secret,
                  seldon_rest_endpoint=f"{args.host}:{args.oauth_port or args.port}",
                  seldon_grpc_endpoint=endpoint)
    else:
        kw.update(gateway_endpoint=endpoint)
    sc = SeldonClient(**kw)
    out = []
    for _ in range(args.n_requests):
        batch = generate_batch(contract, args.batch_size)
        if args.prnt:
            print(f"{'-' * 40}\nSENDING NEW REQUEST:\n{batch}")
        r = sc.predict(data=batch, names=feature_names(contract))
        if args.endpoint == "send-feedback":
            r = sc.feedback(prediction_request=r.request, prediction_response=r.response, reward=1.0)
        if args.prnt:
            print(f"RECEIVED RESPONSE:\n{r.response}\n")
        out.append(r)
    return out


def create_seldon_api_testing_file(data, target: str, output_path: str) -> bool:
    """Write a contract describing ``data``'s columns (``target`` -> targets)."""
    import pandas as pd

    def describe(name: str, col: "pd.Series") -> Dict:
        d: Dict = {"name": str(name)}
        if pd.api.types.is_numeric_dtype(col):
            d["ftype"] = "continuous"
            is_int = pd.api.types.is_integer_dtype(col)
            d["dtype"] = "INTEGER" if is_int else "FLOAT"
            lo, hi = col.min(), col.max()
            if pd.isnull(lo):
                lo, hi = (0, 1) if is_int else (0.0, 1.0)
            d["range"] = [lo.item() if hasattr(lo, "item") else lo, hi.item() if hasattr(hi, "item") else hi]
        else:
            d["ftype"] = "categorical"
            d["values"] = [v.item() if hasattr(v, "item") else v for v in col.unique().tolist()]
        return d

    contract = {"features": [describe(c, data[c]) for c in data.columns if c != target],
                "targets": [describe(c, data[c]) for c in data.columns if c == target]}
    with open(output_path, "w") as f:
        json.dump(contract, f)
    return True


def _common(p: argparse.ArgumentParser) -> None:
    p.add_argument("contract", type=str, help="File that contains the data contract")
    p.add_argument("host", type=str)
    p.add_argument("port", type=int)
    p.add_argument("--endpoint", choices=["predict", "send-feedback"], default="predict")
    p.add_argument("-b", "--batch-size", type=int, default=1)
    p.add_argument("-n", "--n-requests", type=int, default=1)
    p.add_argument("--grpc", action="store_true")
    p.add_argument("-t", "--tensor", action="store_true")
    p.add_argument("-p", "--prnt", action="store_true", help="Prints requests and responses")
    p.add_argument("--log-level", choices=["DEBUG", "INFO", "ERROR"], default="ERROR")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-tester")
    sub = ap.add_subparsers(dest="cmd", required=True)
    m = sub.add_parser("micro", help="test a microservice's internal API")
    _common(m)
    a = sub.add_parser("api", help="test a deployment's external API")
    _common(a)
    a.add_argument("deployment", type=str, nargs="?", default="mymodel")
    a.add_argument("--namespace", type=str)
    a.add_argument("--oauth-port", type=int)
    a.add_argument("--oauth-key")
    a.add_argument("--oauth-secret")
    args = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, args.log_level))
    res = run_microservice(args) if args.cmd == "micro" else run_api(args)
    return 0 if all(r.success for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
