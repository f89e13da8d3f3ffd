// Generates tests/golden/chacha20_openssl.json: ChaCha20 keystream words from
// OpenSSL (node crypto 'chacha20', IV = 32-bit LE counter || 96-bit nonce).
// With nonce = 0 and counter < 2^32 this equals rand_chacha's layout
// (64-bit counter in words 12-13, stream 0 in words 14-15), so it pins the
// oracle's ChaCha core (rounds = 20; StdRng then runs the same core at 12).
// Usage: node tests/golden/make_chacha_fixture.js > tests/golden/chacha20_openssl.json
const crypto = require('crypto');
const cases = [];
const keys = [
  Buffer.alloc(32, 0),
  Buffer.from([...Array(32).keys()]),
  Buffer.from('3f1c0a7799f2b0e44d6e21c8a9b53372d1e04f6a8b9c0d1e2f30415263748596', 'hex'),
];
const counters = [0, 1, 7, 1000003];
for (const key of keys) {
  for (const ctr of counters) {
    const iv = Buffer.alloc(16, 0);
    iv.writeUInt32LE(ctr, 0);
    const c = crypto.createCipheriv('chacha20', key, iv);
    const ks = c.update(Buffer.alloc(64 * 3, 0));
    const words = [];
    for (let i = 0; i < ks.length; i += 4) words.push(ks.readUInt32LE(i));
    const kw = [];
    for (let i = 0; i < 32; i += 4) kw.push(key.readUInt32LE(i));
    cases.push({ key_words: kw, counter: ctr, words });
  }
}
process.stdout.write(JSON.stringify({ source: 'node ' + process.version + ' OpenSSL chacha20', cases }, null, 0) + '\n');
