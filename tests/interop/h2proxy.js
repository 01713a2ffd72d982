// An independent HTTP/2 front end for the interop tests (tests/test_http2_interop.py): Node's `http2` module
// (nghttp2 underneath) terminating HTTP/2 — cleartext prior knowledge, or TLS with ALPN "h2" — and forwarding
// every stream to a fake apiserver over HTTP/1.1, response bodies (watch streams included) piped as they
// arrive.  Its SETTINGS are deliberately tighter than a kube-apiserver's: 50 concurrent streams and a 64 KiB
// initial window, so the clients' stream limits and flow control are exercised by another implementation.
//
//   node h2proxy.js <upstream http://host:port> <h2c|tls> [cert key]
// prints {"port": N} once listening; a line "goaway" on stdin sends GOAWAY(NO_ERROR) on every open session
// and answers {"goaway": <sessions>}; "stats" answers {"streams": N, "sessions": N}.
'use strict';
const http2 = require('http2');
const http = require('http');
const fs = require('fs');

const [, , upstream, mode, certFile, keyFile] = process.argv;
const up = new URL(upstream);
const settings = { maxConcurrentStreams: 50, initialWindowSize: 65535 };
const sessions = new Set();
let streams = 0;
let open = 0;
const HOP = new Set(['connection', 'keep-alive', 'proxy-connection', 'transfer-encoding', 'upgrade', 'te']);

function onStream(stream, headers) {
  streams += 1;
  open += 1;
  stream.on('close', () => { open -= 1; });
  const fwd = {};
  for (const [k, v] of Object.entries(headers)) {
    if (!k.startsWith(':') && !HOP.has(k)) fwd[k] = v;
  }
  fwd.host = up.host;
  const req = http.request({ host: up.hostname, port: up.port, method: headers[':method'], path: headers[':path'],
                             headers: fwd }, (res) => {
    const out = { ':status': res.statusCode };
    for (const k of ['content-type', 'retry-after', 'content-length']) {
      if (res.headers[k] !== undefined) out[k] = res.headers[k];
    }
    if (stream.destroyed) { res.destroy(); return; }
    stream.respond(out);
    res.pipe(stream);
  });
  req.on('error', () => {
    if (!stream.destroyed && !stream.headersSent) {
      stream.respond({ ':status': 502 });
      stream.end();
    }
  });
  stream.on('close', () => req.destroy());  // the client reset (or finished) the stream: drop the upstream request
  stream.on('error', () => req.destroy());
  stream.pipe(req);
}

const server = mode === 'tls'
  ? http2.createSecureServer({ key: fs.readFileSync(keyFile), cert: fs.readFileSync(certFile), settings, maxSessionMemory: 64,
                                allowHTTP1: false })
  : http2.createServer({ settings, maxSessionMemory: 64 });
server.on('stream', onStream);
server.on('session', (s) => {
  sessions.add(s);
  s.on('close', () => sessions.delete(s));
  s.on('error', () => {});
});
server.listen(0, '127.0.0.1', () => {
  process.stdout.write(JSON.stringify({ port: server.address().port }) + '\n');
});
process.stdin.setEncoding('utf8');
process.stdin.on('data', (d) => {
  for (const line of d.split('\n')) {
    if (line.trim() === 'goaway') {
      const n = sessions.size;
      for (const s of sessions) s.goaway(0);
      process.stdout.write(JSON.stringify({ goaway: n }) + '\n');
    } else if (line.trim() === 'stats') {
      process.stdout.write(JSON.stringify({ streams, open, sessions: sessions.size }) + '\n');
    }
  }
});
process.stdin.on('end', () => process.exit(0));
