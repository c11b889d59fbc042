import io.seldon.amd.wrapper.SeldonComponent;
import java.util.Arrays;
import java.util.List;
import java.util.Map;

/** Test model (reference wrappers/s2i/java/test/model-template-app ExampleModelHandler). */
public class ExampleModel implements SeldonComponent {
  private final double weight;

  public ExampleModel(Map<String, Object> params) {
    Object w = params.get("weight");
    this.weight = w instanceof Number ? ((Number) w).doubleValue() : 1.0;
  }

  @Override
  public double[][] predict(double[][] x, List<String> names) {
    double[][] out = new double[x.length][2];
    for (int r = 0; r < x.length; r++) {
      double s = 0;
      for (double v : x[r]) s += weight * v;
      double p = 1.0 / (1.0 + Math.exp(-s));
      out[r][0] = 1 - p;
      out[r][1] = p;
    }
    return out;
  }

  @Override
  public List<String> classNames() {
    return Arrays.asList("neg", "pos");
  }
}
