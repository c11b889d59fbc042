# Test model (reference wrappers/s2i/R/test/model-template-app/MyModel.R):
# a fixed linear scorer over the request columns.
initialise_seldon <- function(params) {
  w <- if (is.null(params$weight)) 1 else params$weight
  structure(list(weight = w), class = "mymodel")
}

predict.mymodel <- function(obj, newdata = list()) {
  s <- as.matrix(newdata) %*% rep(obj$weight, ncol(newdata))
  p <- 1 / (1 + exp(-s))
  out <- cbind(1 - p, p)
  colnames(out) <- c("neg", "pos")
  out
}

send_feedback.mymodel <- function(obj, request = list(), reward = 1, truth = NULL, routing = NULL) {
  invisible(NULL)
}
