package io.seldon.amd.wrapper;

import java.util.Collections;
import java.util.List;
import java.util.Map;

/**
 * A Java graph component (SURVEY P1; reference wrappers/s2i/java + the
 * seldon-core-wrapper library's SeldonPredictionService).  Implement the
 * methods the node's type needs; rows arrive as double[rows][cols] with the
 * request's column names.  Constructors may take a {@code Map<String,Object>}
 * of the typed PREDICTIVE_UNIT_PARAMETERS.
 */
public interface SeldonComponent {
  default double[][] predict(double[][] x, List<String> names) {
    throw new UnsupportedOperationException("predict is not implemented");
  }

  default double[][] transformInput(double[][] x, List<String> names) {
    return x;
  }

  default double[][] transformOutput(double[][] x, List<String> names) {
    return x;
  }

  /** Branch index for a ROUTER node; -1 sends the request to every child. */
  default int route(double[][] x, List<String> names) {
    throw new UnsupportedOperationException("route is not implemented");
  }

  default double[][] aggregate(List<double[][]> xs, List<List<String>> names) {
    throw new UnsupportedOperationException("aggregate is not implemented");
  }

  default void sendFeedback(double[][] x, List<String> names, double reward, double[][] truth, Integer routing) {}

  /** Output column names (default t:0 .. t:C-1, as the Python wrapper). */
  default List<String> classNames() {
    return Collections.emptyList();
  }

  default Map<String, Object> tags() {
    return Collections.emptyMap();
  }

  /** Custom metrics: maps with "type" (COUNTER|GAUGE|TIMER), "key", "value". */
  default List<Map<String, Object>> metrics() {
    return Collections.emptyList();
  }
}
