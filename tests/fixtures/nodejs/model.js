// Test component for the NodeJS wrapper (wrappers/nodejs/microservice.js):
// predict doubles every value (scaled by the `scale` parameter), route picks
// child 1 when the first feature is > 0, aggregate averages the inputs,
// feedback is recorded and echoed through tags.
class DoublerModel {
  constructor(params) {
    this.scale = params.scale === undefined ? 2 : params.scale;
    this.feedback = 0;
    this.ready = false;
  }
  async init() {
    this.ready = true;
  }
  predict(X, names) {
    const f = (v) => (Array.isArray(v) ? v.map(f) : v * this.scale);
    return f(X);
  }
  route(X) {
    return X[0][0] > 0 ? 1 : 0;
  }
  aggregate(Xs) {
    const n = Xs.length;
    return Xs[0].map((row, i) => row.map((_, j) => Xs.reduce((s, x) => s + x[i][j], 0) / n));
  }
  transform_output(X) {
    return Promise.resolve(X.map((r) => r.map((v) => v + 1)));
  }
  send_feedback(X, names, reward, truth) {
    this.feedback += 1;
    this.lastReward = reward;
  }
  tags() {
    return { ready: this.ready, feedback: this.feedback };
  }
  metrics() {
    return [{ type: "COUNTER", key: "node_requests", value: 1 }];
  }
}
module.exports = DoublerModel;
