// Generates Poseidon known-answer vectors by running the REFERENCE's own JS
// Poseidon (test/poseidon.js:134-137) in this container. Output is committed as
// tests/golden/poseidon_kats.json; the reference never travels to the GPU box.
//   node tools/gen_poseidon_kats.js /root/reference/test/poseidon.js tests/golden/poseidon_kats.json
// Inputs: SURVEY.md §8d config 1 — KATs (0,0), (1,2), (p-1,p-1) and pairs drawn
// uniformly in [0,p) from SplitMix64 seed 0x1 (4 x u64 little-endian words,
// rejection-sampled < p); plus smaller random sets for n = 1,3,4,5 (seed 0x11..).
const fs = require('fs');
const path = require('path');
const { poseidon } = require(path.resolve(process.argv[2]));
const out = process.argv[3];
const P = 21888242871839275222246405745257275088548364400416034343698204186575808495617n;
const M64 = (1n << 64n) - 1n;
function splitmix(seed) {
  let s = BigInt(seed) & M64;
  return () => {
    s = (s + 0x9E3779B97F4A7C15n) & M64;
    let z = s;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M64;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M64;
    return z ^ (z >> 31n);
  };
}
function frSampler(seed) {
  const nx = splitmix(seed);
  return () => {
    for (;;) {
      const x = nx() | (nx() << 64n) | (nx() << 128n) | (nx() << 192n);
      if (x < P) return x;
    }
  };
}
const cases = [];
const add = (ins) => cases.push({ in: ins.map(String), out: poseidon(ins).toString() });
add([0n, 0n]); add([1n, 2n]); add([P - 1n, P - 1n]);
let r = frSampler(1);
const NPAIRS = parseInt(process.env.NPAIRS || '1000', 10);
for (let i = 0; i < NPAIRS; i++) add([r(), r()]);
add([1n]); add([1n, 2n, 3n]); add([1n, 2n, 3n, 4n]); add([1n, 2n, 3n, 4n, 5n]);
for (const n of [1, 3, 4, 5]) {
  r = frSampler(0x10 + n);
  for (let i = 0; i < 50; i++) { const v = []; for (let k = 0; k < n; k++) v.push(r()); add(v); }
}
fs.writeFileSync(out, JSON.stringify({ generator: 'reference test/poseidon.js via tools/gen_poseidon_kats.js', cases }, null, 0));
console.log('wrote', cases.length, 'cases to', out);
