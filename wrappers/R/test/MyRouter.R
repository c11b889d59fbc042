# Test router (reference wrappers/s2i/R/test/router-template-app/MyRouter.R).
initialise_seldon <- function(params) structure(list(), class = "myrouter")

route.myrouter <- function(obj, data = list()) {
  if (sum(as.matrix(data)) > 0) 1L else 0L
}

send_feedback.myrouter <- function(obj, request = list(), reward = 1, truth = NULL, routing = NULL) {
  invisible(NULL)
}
