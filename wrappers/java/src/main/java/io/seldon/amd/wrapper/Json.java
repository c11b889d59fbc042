package io.seldon.amd.wrapper;

import java.util.ArrayList;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

/** Minimal JSON reader/writer (objects -> LinkedHashMap, arrays -> ArrayList, numbers -> Double). */
public final class Json {
  private final String s;
  private int i;

  private Json(String s) {
    this.s = s;
  }

  public static Object parse(String text) {
    Json p = new Json(text);
    p.ws();
    Object v = p.value();
    p.ws();
    if (p.i != p.s.length()) throw new IllegalArgumentException("trailing characters at " + p.i);
    return v;
  }

  private void ws() {
    while (i < s.length() && Character.isWhitespace(s.charAt(i))) i++;
  }

  private char peek() {
    if (i >= s.length()) throw new IllegalArgumentException("unexpected end of JSON");
    return s.charAt(i);
  }

  private void expect(char c) {
    if (peek() != c) throw new IllegalArgumentException("expected '" + c + "' at " + i);
    i++;
  }

  private Object value() {
    char c = peek();
    switch (c) {
      case '{': return object();
      case '[': return array();
      case '"': return string();
      case 't': lit("true"); return Boolean.TRUE;
      case 'f': lit("false"); return Boolean.FALSE;
      case 'n': lit("null"); return null;
      default: return number();
    }
  }

  private void lit(String w) {
    if (!s.startsWith(w, i)) throw new IllegalArgumentException("bad literal at " + i);
    i += w.length();
  }

  private Map<String, Object> object() {
    Map<String, Object> m = new LinkedHashMap<>();
    expect('{');
    ws();
    if (peek() == '}') { i++; return m; }
    while (true) {
      ws();
      String k = string();
      ws();
      expect(':');
      ws();
      m.put(k, value());
      ws();
      if (peek() == ',') { i++; continue; }
      expect('}');
      return m;
    }
  }

  private List<Object> array() {
    List<Object> a = new ArrayList<>();
    expect('[');
    ws();
    if (peek() == ']') { i++; return a; }
    while (true) {
      ws();
      a.add(value());
      ws();
      if (peek() == ',') { i++; continue; }
      expect(']');
      return a;
    }
  }

  private String string() {
    expect('"');
    StringBuilder b = new StringBuilder();
    while (true) {
      char c = s.charAt(i++);
      if (c == '"') return b.toString();
      if (c != '\\') { b.append(c); continue; }
      char e = s.charAt(i++);
      switch (e) {
        case 'n': b.append('\n'); break;
        case 't': b.append('\t'); break;
        case 'r': b.append('\r'); break;
        case 'b': b.append('\b'); break;
        case 'f': b.append('\f'); break;
        case 'u': b.append((char) Integer.parseInt(s.substring(i, i + 4), 16)); i += 4; break;
        default: b.append(e);
      }
    }
  }

  private Double number() {
    int st = i;
    while (i < s.length() && "+-0123456789.eE".indexOf(s.charAt(i)) >= 0) i++;
    if (st == i) throw new IllegalArgumentException("unexpected character at " + i);
    return Double.valueOf(s.substring(st, i));
  }

  public static String write(Object v) {
    StringBuilder b = new StringBuilder();
    write(b, v);
    return b.toString();
  }

  @SuppressWarnings("unchecked")
  private static void write(StringBuilder b, Object v) {
    if (v == null) {
      b.append("null");
    } else if (v instanceof String) {
      b.append('"');
      for (char c : ((String) v).toCharArray()) {
        if (c == '"' || c == '\\') b.append('\\').append(c);
        else if (c < 0x20) b.append(String.format("\\u%04x", (int) c));
        else b.append(c);
      }
      b.append('"');
    } else if (v instanceof Double || v instanceof Float) {
      double d = ((Number) v).doubleValue();
      if (d == Math.rint(d) && Math.abs(d) < 1e15) b.append((long) d).append(".0");
      else b.append(Double.toString(d));
    } else if (v instanceof Number || v instanceof Boolean) {
      b.append(v);
    } else if (v instanceof Map) {
      b.append('{');
      boolean first = true;
      for (Map.Entry<String, Object> e : ((Map<String, Object>) v).entrySet()) {
        if (!first) b.append(',');
        first = false;
        write(b, e.getKey());
        b.append(':');
        write(b, e.getValue());
      }
      b.append('}');
    } else if (v instanceof double[][]) {
      b.append('[');
      double[][] m = (double[][]) v;
      for (int r = 0; r < m.length; r++) {
        if (r > 0) b.append(',');
        write(b, m[r]);
      }
      b.append(']');
    } else if (v instanceof double[]) {
      b.append('[');
      double[] a = (double[]) v;
      for (int c = 0; c < a.length; c++) {
        if (c > 0) b.append(',');
        write(b, a[c]);
      }
      b.append(']');
    } else if (v instanceof Iterable) {
      b.append('[');
      boolean first = true;
      for (Object o : (Iterable<Object>) v) {
        if (!first) b.append(',');
        first = false;
        write(b, o);
      }
      b.append(']');
    } else {
      write(b, v.toString());
    }
  }
}
