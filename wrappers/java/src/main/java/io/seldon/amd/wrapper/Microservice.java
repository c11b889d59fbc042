package io.seldon.amd.wrapper;

import com.sun.net.httpserver.HttpExchange;
import com.sun.net.httpserver.HttpServer;
import java.io.ByteArrayOutputStream;
import java.io.IOException;
import java.io.InputStream;
import java.io.OutputStream;
import java.lang.reflect.Constructor;
import java.net.InetSocketAddress;
import java.net.URLDecoder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.HashMap;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.concurrent.Executors;

/**
 * Seldon microservice for Java components (SURVEY P1; reference
 * wrappers/s2i/java/s2i/bin/run launching a Spring Boot app on the
 * seldon-core-wrapper library).  JDK only: com.sun.net.httpserver serves the
 * internal REST API the engine calls for remote nodes
 * (csrc/server/remote_unit.cc; engine InternalPredictionService.java:364-453):
 *
 * <pre>
 *   POST/GET /predict /send-feedback              (MODEL)
 *            /route /send-feedback                (ROUTER)
 *            /transform-input /transform-output   (TRANSFORMER)
 *            /aggregate                           (COMBINER)
 *   GET      /health/ping /health/status /ready /live
 * </pre>
 *
 * The SeldonMessage comes as a form field {@code json=}, a {@code json} query
 * parameter, or a raw JSON body; replies keep the request's data kind.
 *
 * <pre>java -cp app.jar:wrapper.jar io.seldon.amd.wrapper.Microservice com.example.MyModel --service MODEL</pre>
 *
 * No JVM exists in the build image, so parity with the reference is unpinned;
 * tests/test_wrappers.py pins routes and message rules statically.
 */
public final class Microservice {
  static final Map<String, List<String>> ROUTES = new HashMap<>();

  static {
    ROUTES.put("MODEL", Arrays.asList("/predict", "/send-feedback"));
    ROUTES.put("ROUTER", Arrays.asList("/route", "/send-feedback"));
    ROUTES.put("TRANSFORMER", Arrays.asList("/transform-input", "/transform-output"));
    ROUTES.put("OUTPUT_TRANSFORMER", Arrays.asList("/transform-input", "/transform-output"));
    ROUTES.put("COMBINER", Arrays.asList("/aggregate"));
  }

  private final SeldonComponent component;
  private final String service;

  Microservice(SeldonComponent component, String service) {
    this.component = component;
    this.service = service;
  }

  // ---------------------------------------------------------- parameters
  static Map<String, Object> typedParameters(String json) {
    Map<String, Object> out = new LinkedHashMap<>();
    if (json == null || json.trim().isEmpty()) return out;
    for (Object o : (List<?>) Json.parse(json)) {
      Map<?, ?> p = (Map<?, ?>) o;
      String name = String.valueOf(p.get("name"));
      String value = String.valueOf(p.get("value"));
      String type = p.get("type") == null ? "STRING" : String.valueOf(p.get("type")).toUpperCase();
      switch (type) {
        case "INT": out.put(name, Integer.parseInt(value)); break;
        case "FLOAT":
        case "DOUBLE": out.put(name, Double.parseDouble(value)); break;
        case "BOOL": out.put(name, Boolean.parseBoolean(value) || value.equals("1")); break;
        default: out.put(name, value);
      }
    }
    return out;
  }

  static SeldonComponent load(String className, Map<String, Object> params) throws Exception {
    Class<?> cls = Class.forName(className);
    for (Constructor<?> c : cls.getConstructors()) {
      Class<?>[] t = c.getParameterTypes();
      if (t.length == 1 && t[0].isAssignableFrom(Map.class)) return (SeldonComponent) c.newInstance(params);
    }
    return (SeldonComponent) cls.getConstructor().newInstance();
  }

  // ------------------------------------------------------------ payloads
  static final class Data {
    double[][] x;
    List<String> names = new ArrayList<>();
    String kind = "ndarray";
  }

  @SuppressWarnings("unchecked")
  static Data decode(Map<String, Object> msg) {
    Map<String, Object> d = (Map<String, Object>) msg.get("data");
    if (d == null) throw new IllegalArgumentException("Request has no data field");
    Data out = new Data();
    if (d.get("names") instanceof List) for (Object n : (List<?>) d.get("names")) out.names.add(String.valueOf(n));
    if (d.get("tensor") instanceof Map) {
      Map<String, Object> t = (Map<String, Object>) d.get("tensor");
      List<?> shape = (List<?>) t.get("shape");
      List<?> vals = (List<?>) t.get("values");
      int rows = shape.size() >= 2 ? ((Number) shape.get(0)).intValue() : 1;
      int cols = rows == 0 ? 0 : vals.size() / rows;
      out.x = new double[rows][cols];
      for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) out.x[r][c] = ((Number) vals.get(r * cols + c)).doubleValue();
      out.kind = "tensor";
    } else if (d.get("ndarray") instanceof List) {
      List<?> rows = (List<?>) d.get("ndarray");
      boolean flat = !rows.isEmpty() && !(rows.get(0) instanceof List);
      if (flat) rows = Arrays.asList(rows);
      out.x = new double[rows.size()][];
      for (int r = 0; r < rows.size(); r++) {
        List<?> row = (List<?>) rows.get(r);
        out.x[r] = new double[row.size()];
        for (int c = 0; c < row.size(); c++) out.x[r][c] = ((Number) row.get(c)).doubleValue();
      }
    } else {
      throw new IllegalArgumentException("data field must contain ndarray or tensor field");
    }
    return out;
  }

  @SuppressWarnings("unchecked")
  String encode(Map<String, Object> request, String kind, double[][] y) {
    List<String> names = component.classNames();
    int cols = y.length == 0 ? 0 : y[0].length;
    if (names.size() != cols) {
      names = new ArrayList<>();
      for (int c = 0; c < cols; c++) names.add("t:" + c);
    }
    Map<String, Object> data = new LinkedHashMap<>();
    data.put("names", names);
    if (kind.equals("tensor")) {
      Map<String, Object> t = new LinkedHashMap<>();
      t.put("shape", Arrays.asList(y.length, cols));
      double[] flat = new double[y.length * cols];
      for (int r = 0; r < y.length; r++) System.arraycopy(y[r], 0, flat, r * cols, cols);
      t.put("values", flat);
      data.put("tensor", t);
    } else {
      data.put("ndarray", y);
    }
    Map<String, Object> out = new LinkedHashMap<>();
    Map<String, Object> meta = new LinkedHashMap<>();
    Object reqMeta = request.get("meta");
    if (reqMeta instanceof Map && ((Map<String, Object>) reqMeta).get("puid") != null)
      meta.put("puid", ((Map<String, Object>) reqMeta).get("puid"));
    if (!component.tags().isEmpty()) meta.put("tags", component.tags());
    if (!component.metrics().isEmpty()) meta.put("metrics", component.metrics());
    if (!meta.isEmpty()) out.put("meta", meta);
    out.put("data", data);
    return Json.write(out);
  }

  static String formField(String s, String key) {
    if (s == null || s.isEmpty()) return null;
    for (String kv : s.split("&")) {
      int eq = kv.indexOf('=');
      String k = URLDecoder.decode(eq < 0 ? kv : kv.substring(0, eq), StandardCharsets.UTF_8);
      if (k.equals(key)) return eq < 0 ? "" : URLDecoder.decode(kv.substring(eq + 1), StandardCharsets.UTF_8);
    }
    return null;
  }

  static String requestJson(String body, String query, String contentType) {
    String j = null;
    if (!body.isEmpty() && (contentType == null || !contentType.contains("json"))) j = formField(body, "json");
    if (j == null) j = formField(query, "json");
    if (j == null && !body.isEmpty()) j = body;
    if (j == null) throw new IllegalArgumentException("Empty json parameter in data");
    return j;
  }

  // ------------------------------------------------------------ handlers
  @SuppressWarnings("unchecked")
  String handle(String path, String json) {
    Map<String, Object> msg = (Map<String, Object>) Json.parse(json);
    switch (path) {
      case "/predict": {
        Data d = decode(msg);
        return encode(msg, d.kind, component.predict(d.x, d.names));
      }
      case "/transform-input": {
        Data d = decode(msg);
        return encode(msg, d.kind, component.transformInput(d.x, d.names));
      }
      case "/transform-output": {
        Data d = decode(msg);
        return encode(msg, d.kind, component.transformOutput(d.x, d.names));
      }
      case "/route": {
        Data d = decode(msg);
        return encode(msg, d.kind, new double[][] {{component.route(d.x, d.names)}});
      }
      case "/aggregate": {
        List<?> parts = (List<?>) msg.get("seldonMessages");
        if (parts == null || parts.isEmpty()) throw new IllegalArgumentException("aggregate expects seldonMessages");
        List<double[][]> xs = new ArrayList<>();
        List<List<String>> names = new ArrayList<>();
        String kind = "ndarray";
        for (Object p : parts) {
          Data d = decode((Map<String, Object>) p);
          xs.add(d.x);
          names.add(d.names);
          kind = d.kind;
        }
        return encode((Map<String, Object>) parts.get(0), kind, component.aggregate(xs, names));
      }
      case "/send-feedback": {
        Map<String, Object> req = (Map<String, Object>) msg.get("request");
        if (req == null) throw new IllegalArgumentException("request field is missing");
        Data d = decode(req);
        double reward = msg.get("reward") instanceof Number ? ((Number) msg.get("reward")).doubleValue() : 0.0;
        double[][] truth = msg.get("truth") instanceof Map ? decode((Map<String, Object>) msg.get("truth")).x : null;
        component.sendFeedback(d.x, d.names, reward, truth, null);
        return "{}";
      }
      default:
        throw new IllegalArgumentException("unknown path " + path);
    }
  }

  void serve(int port) throws IOException {
    HttpServer srv = HttpServer.create(new InetSocketAddress("0.0.0.0", port), 256);
    srv.createContext("/", this::exchange);
    srv.setExecutor(Executors.newFixedThreadPool(Math.max(2, Runtime.getRuntime().availableProcessors())));
    srv.start();
    System.out.println("Java " + service + " microservice on :" + port);
  }

  private void exchange(HttpExchange ex) throws IOException {
    String path = ex.getRequestURI().getPath();
    int status = 200;
    String body;
    try {
      if (path.equals("/health/ping") || path.equals("/ping")) {
        body = "\"pong\"";
      } else if (path.equals("/health/status") || path.equals("/ready") || path.equals("/live")) {
        body = "{\"status\":\"ok\"}";
      } else if (!ROUTES.get(service).contains(path)) {
        status = 404;
        body = "{\"error\":\"not found\"}";
      } else {
        String raw = readAll(ex.getRequestBody());
        body = handle(path, requestJson(raw, ex.getRequestURI().getRawQuery(),
                                        ex.getRequestHeaders().getFirst("Content-Type")));
      }
    } catch (RuntimeException e) {
      status = 400;
      Map<String, Object> st = new LinkedHashMap<>();
      st.put("status", 1);
      st.put("info", String.valueOf(e.getMessage()));
      st.put("code", -1);
      st.put("reason", "MICROSERVICE_BAD_DATA");
      body = Json.write(Map.of("status", st));
    }
    byte[] out = body.getBytes(StandardCharsets.UTF_8);
    ex.getResponseHeaders().set("Content-Type", "application/json");
    ex.sendResponseHeaders(status, out.length);
    try (OutputStream os = ex.getResponseBody()) {
      os.write(out);
    }
  }

  private static String readAll(InputStream in) throws IOException {
    ByteArrayOutputStream b = new ByteArrayOutputStream();
    byte[] buf = new byte[8192];
    int n;
    while ((n = in.read(buf)) > 0) b.write(buf, 0, n);
    return b.toString(StandardCharsets.UTF_8);
  }

  public static void main(String[] args) throws Exception {
    String cls = null, service = "MODEL", api = "REST";
    String params = System.getenv().getOrDefault("PREDICTIVE_UNIT_PARAMETERS", "[]");
    for (int i = 0; i < args.length; i++) {
      switch (args[i]) {
        case "--service": service = args[++i].toUpperCase(); break;
        case "--api": api = args[++i].toUpperCase(); break;
        case "--parameters": params = args[++i]; break;
        default: if (cls == null) cls = args[i];
      }
    }
    if (cls == null) throw new IllegalArgumentException("usage: Microservice <ComponentClass> [--service TYPE]");
    if (!ROUTES.containsKey(service)) throw new IllegalArgumentException("Invalid service type [" + service + "]");
    if (!api.equals("REST")) throw new IllegalArgumentException("Invalid API type [" + api + "]: REST only");
    int port = Integer.parseInt(System.getenv().getOrDefault("PREDICTIVE_UNIT_SERVICE_PORT", "5000"));
    new Microservice(load(cls, typedParameters(params)), service).serve(port);
  }
}
