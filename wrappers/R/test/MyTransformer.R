# Test transformer (reference wrappers/s2i/R/test/transformer-template-app/MyTransformer.R):
# min-max scaling of the whole request, as examples/transformers/mean_transformer.
initialise_seldon <- function(params) structure(list(), class = "mytransformer")

transform_input.mytransformer <- function(obj, newdata = list()) {
  m <- as.matrix(newdata)
  r <- max(m) - min(m)
  out <- if (r == 0) m * 0 else (m - min(m)) / r
  colnames(out) <- colnames(newdata)
  out
}
