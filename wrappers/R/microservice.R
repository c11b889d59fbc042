#!/usr/bin/env Rscript
# Seldon microservice wrapper for R components (SURVEY P1; reference
# wrappers/s2i/R/microservice.R:129-304).  Serves a user model over the
# internal REST API the engine calls for remote graph nodes
# (csrc/server/remote_unit.cc, engine InternalPredictionService.java:364-453):
#
#   POST/GET /predict /send-feedback          (--service MODEL)
#            /route /send-feedback            (--service ROUTER)
#            /transform-input /transform-output (--service TRANSFORMER)
#            /aggregate                       (--service COMBINER)
#   GET      /health/ping /health/status /ready /live
#
# The SeldonMessage arrives as a form field `json=`, a `json` query
# parameter, or a raw JSON body; the reply keeps the request's data kind
# (ndarray stays ndarray, tensor stays tensor), as the Python wrapper does
# (python/seldon_core/utils.py construct_response_json).
#
# User component, an R file defining
#   initialise_seldon(params)               -> object with an S3 class
#   predict.<class>(obj, newdata)           -> matrix / data.frame
#   transform_input.<class>(obj, newdata)   -> matrix / data.frame (identity if absent)
#   transform_output.<class>(obj, newdata)  -> matrix / data.frame (identity if absent)
#   route.<class>(obj, data)                -> integer branch (-1 = all children)
#   aggregate.<class>(obj, datas)           -> matrix (list of the children's frames)
#   send_feedback.<class>(obj, request, reward, truth, routing)
#   tags.<class>(obj) -> named list,  metrics.<class>(obj) -> list(list(type, key, value))
# Parameters come from --parameters or PREDICTIVE_UNIT_PARAMETERS (JSON
# [{name, value, type}] with type INT | FLOAT | DOUBLE | STRING | BOOL).
#
# Dependencies: httpuv and jsonlite only (no plumber / optparse / urltools /
# stringi as in the reference).  No R runtime exists in the build image, so
# parity with the reference wrapper is unpinned; tests/test_wrappers.py pins
# the routes, option names and message rules statically.

suppressPackageStartupMessages({
  library(httpuv)
  library(jsonlite)
})

# ------------------------------------------------------------------ options
parse_cli <- function(argv) {
  opts <- list(model = "", api = "REST", service = "MODEL", persistence = 0L,
               parameters = Sys.getenv("PREDICTIVE_UNIT_PARAMETERS", "[]"))
  i <- 1
  while (i <= length(argv)) {
    a <- argv[[i]]
    kv <- regmatches(a, regexec("^--?([A-Za-z]+)(=(.*))?$", a))[[1]]
    if (length(kv) == 0) { i <- i + 1; next }
    key <- switch(kv[2], m = "model", a = "api", s = "service", e = "persistence", p = "parameters", kv[2])
    if (nzchar(kv[3])) {
      val <- kv[4]
    } else {
      i <- i + 1
      val <- if (i <= length(argv)) argv[[i]] else ""
    }
    opts[[key]] <- val
    i <- i + 1
  }
  opts$api <- toupper(opts$api)
  opts$service <- toupper(opts$service)
  opts$persistence <- as.integer(opts$persistence)
  if (!nzchar(opts$parameters)) opts$parameters <- "[]"
  opts
}

typed_parameters <- function(json) {
  ps <- fromJSON(json, simplifyVector = FALSE)
  out <- list()
  for (p in ps) {
    v <- p$value
    t <- toupper(if (is.null(p$type)) "STRING" else p$type)
    v <- switch(t,
                INT = as.integer(v),
                FLOAT = as.numeric(v),
                DOUBLE = as.numeric(v),
                BOOL = tolower(as.character(v)) %in% c("true", "1", "yes"),
                as.character(v))
    out[[p$name]] <- v
  }
  out
}

# ------------------------------------------------------------- payloads
url_decode_plus <- function(s) utils::URLdecode(gsub("+", " ", s, fixed = TRUE))

form_field <- function(s, key) {
  if (is.null(s) || !nzchar(s)) return(NULL)
  s <- sub("^\\?", "", s)
  for (kv in strsplit(s, "&", fixed = TRUE)[[1]]) {
    parts <- strsplit(kv, "=", fixed = TRUE)[[1]]
    if (length(parts) >= 1 && url_decode_plus(parts[1]) == key)
      return(if (length(parts) >= 2) url_decode_plus(paste(parts[-1], collapse = "=")) else "")
  }
  NULL
}

request_json <- function(req) {
  body <- if (!is.null(req$rook.input)) rawToChar(req$rook.input$read()) else ""
  ctype <- if (is.null(req$CONTENT_TYPE)) "" else req$CONTENT_TYPE
  j <- NULL
  if (nzchar(body) && !grepl("json", ctype, fixed = TRUE)) j <- form_field(body, "json")
  if (is.null(j)) j <- form_field(req$QUERY_STRING, "json")
  if (is.null(j) && nzchar(body)) j <- body
  if (is.null(j)) stop("Empty json parameter in data")
  fromJSON(j, simplifyVector = TRUE, simplifyMatrix = TRUE)
}

data_kind <- function(msg) {
  d <- msg$data
  if (!is.null(d$tensor)) "tensor" else if (!is.null(d$ndarray)) "ndarray" else NA
}

# DefaultData -> data.frame (tensor values are row-major, like numpy)
to_frame <- function(msg) {
  d <- msg$data
  if (is.null(d)) stop("Request has no data field")
  if (!is.null(d$tensor)) {
    shape <- as.integer(d$tensor$shape)
    vals <- as.numeric(d$tensor$values)
    if (length(shape) < 2) shape <- c(1L, length(vals))
    m <- matrix(vals, nrow = shape[1], ncol = prod(shape[-1]), byrow = TRUE)
  } else if (!is.null(d$ndarray)) {
    m <- d$ndarray
    if (is.null(dim(m))) m <- matrix(m, nrow = 1)
  } else {
    stop("data field must contain ndarray or tensor field")
  }
  df <- as.data.frame(m)
  if (!is.null(d$names) && length(d$names) == ncol(df)) colnames(df) <- d$names
  df
}

to_message <- function(request, result, obj) {
  m <- as.matrix(result)
  names <- colnames(m)
  if (is.null(names)) names <- character(0)
  kind <- data_kind(request)
  data <- list(names = I(names))
  if (!is.na(kind) && kind == "tensor") {
    data$tensor <- list(shape = I(dim(m)), values = I(as.numeric(t(m))))
  } else {
    data$ndarray <- m
  }
  out <- list(data = data)
  meta <- list()
  if (!is.null(request$meta$puid)) meta$puid <- request$meta$puid
  if (exists("tags", mode = "function") && hasMethodFor("tags", obj)) meta$tags <- tags(obj)
  if (exists("metrics", mode = "function") && hasMethodFor("metrics", obj)) meta$metrics <- metrics(obj)
  if (length(meta)) out$meta <- meta
  toJSON(out, auto_unbox = TRUE, digits = NA, matrix = "rowmajor")
}

hasMethodFor <- function(generic, obj) {
  any(vapply(class(obj), function(cl) !is.null(utils::getS3method(generic, cl, optional = TRUE)), logical(1)))
}

reply <- function(status, body) {
  list(status = status, headers = list("Content-Type" = "application/json"), body = body)
}

fail <- function(e) {
  reply(400L, toJSON(list(status = list(status = 1L, info = conditionMessage(e), code = -1L,
                                        reason = "MICROSERVICE_BAD_DATA")), auto_unbox = TRUE))
}

# ------------------------------------------------------------- handlers
handle_predict <- function(obj, req) {
  msg <- request_json(req)
  reply(200L, to_message(msg, predict(obj, newdata = to_frame(msg)), obj))
}

handle_transform <- function(obj, req, which) {
  msg <- request_json(req)
  df <- to_frame(msg)
  res <- if (hasMethodFor(which, obj)) get(which)(obj, newdata = df) else df
  reply(200L, to_message(msg, res, obj))
}

handle_route <- function(obj, req) {
  msg <- request_json(req)
  branch <- as.integer(route(obj, data = to_frame(msg)))
  reply(200L, to_message(msg, matrix(branch, nrow = 1, ncol = 1), obj))
}

handle_aggregate <- function(obj, req) {
  msg <- request_json(req)
  parts <- msg$seldonMessages
  if (is.null(parts)) stop("aggregate expects a SeldonMessageList (seldonMessages)")
  frames <- lapply(seq_len(NROW(parts)), function(i) to_frame(list(data = parts$data[i, , drop = FALSE])))
  first <- list(data = parts$data[1, , drop = FALSE])
  reply(200L, to_message(first, aggregate(obj, datas = frames), obj))
}

handle_feedback <- function(obj, req) {
  fb <- request_json(req)
  if (is.null(fb$request)) stop("request field is missing")
  reward <- if (is.null(fb$reward)) 0 else as.numeric(fb$reward)
  truth <- if (!is.null(fb$truth)) to_frame(fb$truth) else NULL
  routing <- NULL
  if (!is.null(fb$response$meta$routing)) routing <- fb$response$meta$routing
  if (hasMethodFor("send_feedback", obj))
    send_feedback(obj, request = to_frame(fb$request), reward = reward, truth = truth, routing = routing)
  reply(200L, "{}")
}

ROUTES <- list(
  MODEL = c("/predict", "/send-feedback"),
  ROUTER = c("/route", "/send-feedback"),
  TRANSFORMER = c("/transform-input", "/transform-output"),
  OUTPUT_TRANSFORMER = c("/transform-input", "/transform-output"),
  COMBINER = c("/aggregate")
)

dispatch <- function(obj, service, req) {
  path <- req$PATH_INFO
  if (path %in% c("/health/ping", "/ping")) return(reply(200L, "\"pong\""))
  if (path %in% c("/health/status", "/ready", "/live")) return(reply(200L, "{\"status\":\"ok\"}"))
  if (!(path %in% ROUTES[[service]])) return(reply(404L, "{\"error\":\"not found\"}"))
  tryCatch(switch(path,
                  "/predict" = handle_predict(obj, req),
                  "/transform-input" = handle_transform(obj, req, "transform_input"),
                  "/transform-output" = handle_transform(obj, req, "transform_output"),
                  "/route" = handle_route(obj, req),
                  "/aggregate" = handle_aggregate(obj, req),
                  "/send-feedback" = handle_feedback(obj, req)),
           error = fail)
}

# ----------------------------------------------------------------- main
send_feedback <- function(x, ...) UseMethod("send_feedback", x)
route <- function(x, ...) UseMethod("route", x)
transform_input <- function(x, ...) UseMethod("transform_input", x)
transform_output <- function(x, ...) UseMethod("transform_output", x)
tags <- function(x, ...) UseMethod("tags", x)
metrics <- function(x, ...) UseMethod("metrics", x)
# `aggregate` and `predict` are stats generics already

main <- function() {
  opts <- parse_cli(commandArgs(trailingOnly = TRUE))
  if (!(opts$service %in% names(ROUTES))) {
    cat(sprintf("Invalid service type [%s]\n", opts$service))
    quit(status = 1)
  }
  if (opts$api != "REST") {
    cat(sprintf("Invalid API type [%s]: the R wrapper serves REST\n", opts$api))
    quit(status = 1)
  }
  if (!file.exists(opts$model)) {
    cat(sprintf("Model file does not exist [%s]\n", opts$model))
    quit(status = 1)
  }
  source(opts$model)
  obj <- initialise_seldon(typed_parameters(opts$parameters))
  port <- as.integer(Sys.getenv("PREDICTIVE_UNIT_SERVICE_PORT", "5000"))
  cat(sprintf("R %s microservice on :%d\n", opts$service, port))
  runServer("0.0.0.0", port, list(call = function(req) dispatch(obj, opts$service, req)))
}

if (!interactive()) main()
