"""Error types of the component API.

Behaviour mirrors the reference wrapper (python/seldon_core/flask_utils.py:67-82,
python/seldon_core/user_model.py:12-16): a bad request from a component is a
400 with body ``{"status": {"status": 1, "info": msg, "code": -1, "reason": ...}}``,
and a component's own ``model_error_handler`` decides status and body for the
exceptions it registers (python/seldon_core/wrapper.py:22-26).
"""
from __future__ import annotations

import json
from typing import Any, Callable, Dict, List, Optional, Tuple, Type


class SeldonMicroserviceException(Exception):
    status_code = 400

    def __init__(self, message: str, status_code: Optional[int] = None, payload: Optional[Dict[str, Any]] = None,
                 reason: str = "MICROSERVICE_BAD_DATA"):
        super().__init__(message)
        self.message = message
        if status_code is not None:
            self.status_code = status_code
        self.payload = payload
        self.reason = reason

    def to_dict(self) -> Dict[str, Any]:
        body = dict(self.payload or {})
        body["status"] = {"status": 1, "info": self.message, "code": -1, "reason": self.reason}
        return body


class JsonResponse:
    """What :func:`jsonify` returns: a JSON body plus a settable
    ``status_code`` (the two things the reference's handlers touch on a
    ``flask.Response``, test_application_exception_microservice.py:34-38)."""

    def __init__(self, body: Any, status_code: int = 200):
        self.body = body
        self.status_code = status_code

    def get_data(self, as_text: bool = False):
        text = json.dumps(self.body)
        return text if as_text else text.encode()


def jsonify(*args: Any, **kwargs: Any) -> JsonResponse:
    """``flask.jsonify`` look-alike for components written without Flask."""
    if args and kwargs:
        raise TypeError("jsonify() takes either positional or keyword arguments")
    body = kwargs if kwargs else (args[0] if len(args) == 1 else list(args))
    return JsonResponse(body)


class ErrorHandlers:
    """A component's ``model_error_handler`` without Flask: the same decorator
    API as the ``flask.Blueprint`` the reference registers
    (python/seldon_core/wrapper.py:22-26)::

        class MyModel:
            model_error_handler = ErrorHandlers("error_handlers", __name__)

            @model_error_handler.app_errorhandler(MyError)
            def handle(error):
                r = jsonify(error.to_dict())
                r.status_code = error.status_code
                return r

    A real ``flask.Blueprint`` works too (see :func:`component_error_reply`)."""

    def __init__(self, name: str = "error_handlers", import_name: str = "", **_: Any):
        self.name = name
        self.import_name = import_name
        self.handlers: List[Tuple[Type[BaseException], Callable]] = []

    def app_errorhandler(self, exc_type: Type[BaseException]) -> Callable[[Callable], Callable]:
        def deco(fn: Callable) -> Callable:
            self.handlers.append((exc_type, fn))
            return fn

        return deco

    errorhandler = app_errorhandler

    def find(self, exc: BaseException) -> Optional[Callable]:
        """The handler of the closest registered base class (Flask's MRO rule)."""
        for klass in type(exc).__mro__:
            for t, fn in self.handlers:
                if t is klass:
                    return fn
        return None


def _reply_from(rv: Any, default_status: int) -> Tuple[int, str]:
    """A handler's return value -> (status, JSON text): a response object, a
    ``(body, status)`` tuple, or a bare JSON-able body."""
    status = default_status
    if isinstance(rv, tuple):
        rv, status = rv[0], int(rv[1]) if len(rv) > 1 and rv[1] is not None else default_status
    if hasattr(rv, "status_code") and hasattr(rv, "get_data"):
        return int(rv.status_code), rv.get_data(as_text=True)
    if isinstance(rv, (bytes, bytearray)):
        return status, rv.decode()
    if isinstance(rv, str):
        return status, rv
    return status, json.dumps(rv)


def component_error_reply(component: Any, exc: BaseException, cache: Optional[Dict[str, Any]] = None
                          ) -> Optional[Tuple[int, str, str]]:
    """The reference wrapper's error contract for a component's exception
    (python/seldon_core/wrapper.py:22-31, flask_utils.py:67-81):

    1. the component's ``model_error_handler`` (an :class:`ErrorHandlers` or a
       real ``flask.Blueprint`` registered on a private app) if it handles
       the exception's class;
    2. else a :class:`SeldonMicroserviceException`: its ``status_code`` and
       ``to_dict()`` (reason ``MICROSERVICE_BAD_DATA`` / ``..._BAD_METRIC``);
    3. else ``None`` (the engine's plain 203).

    Returns ``(http status, JSON body text, info)``."""
    handler = getattr(component, "model_error_handler", None)
    info = str(getattr(exc, "message", "") or exc)
    if handler is not None:
        if isinstance(handler, ErrorHandlers):
            fn = handler.find(exc)
            if fn is not None:
                return (*_reply_from(fn(exc), int(getattr(exc, "status_code", 500) or 500)), info)
        elif hasattr(handler, "record_once") or hasattr(handler, "deferred_functions"):
            r = _flask_reply(handler, exc, cache if cache is not None else {})
            if r is not None:
                return (*r, info)
        elif isinstance(handler, dict):  # {ExceptionClass: fn}
            for klass in type(exc).__mro__:
                if klass in handler:
                    return (*_reply_from(handler[klass](exc), int(getattr(exc, "status_code", 500) or 500)), info)
    if isinstance(exc, SeldonMicroserviceException):
        return int(exc.status_code), json.dumps(exc.to_dict()), info
    return None


def _flask_reply(blueprint: Any, exc: BaseException, cache: Dict[str, Any]) -> Optional[Tuple[int, str]]:
    try:
        import flask
    except ImportError:
        return None
    app = cache.get("flask_app")
    if app is None:
        app = flask.Flask("seldon_core_amd_error_handlers")
        app.register_blueprint(blueprint)
        cache["flask_app"] = app
    if not isinstance(exc, Exception):
        return None
    with app.test_request_context():
        try:
            rv = app.handle_user_exception(exc)
        except BaseException:  # no handler for this class: Flask re-raises it
            return None
        resp = app.make_response(rv)
        return int(resp.status_code), resp.get_data(as_text=True)


class SeldonNotImplementedError(SeldonMicroserviceException):
    """Raised by the optional methods of :class:`SeldonComponent`."""

    status_code = 400

    def __init__(self, message: str):
        super().__init__(message)


class EngineError(RuntimeError):
    """A native-engine error (``Status{code 20x, reason, info}``)."""

    def __init__(self, http_status: int, body: Dict[str, Any]):
        self.http_status = http_status
        self.body = body
        super().__init__(f"{http_status}: {body}")
