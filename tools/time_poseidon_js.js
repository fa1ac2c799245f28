// Config 1 reference point (SURVEY.md §8d): times the REFERENCE's own JS PoseidonHash (test/poseidon.js:134-137,
// PoseidonEx with every Sigma / Mix / MixLast intermediate — the values circom's PoseidonHash(2) witness holds) on
// config 1's 1,003 input pairs, one thread, in this container (the reference never travels to the GPU box).
//   node tools/time_poseidon_js.js /root/reference/test/poseidon.js profiles/r5_config1/poseidon_js.json
const fs = require('fs');
const os = require('os');
const path = require('path');
const { poseidon } = require(path.resolve(process.argv[2]));
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
const nx = splitmix(1);
const fr = () => { for (;;) { const x = nx() | (nx() << 64n) | (nx() << 128n) | (nx() << 192n); if (x < P) return x; } };
const pairs = [[0n, 0n], [1n, 2n], [P - 1n, P - 1n]];
for (let i = 0; i < 1000; i++) pairs.push([fr(), fr()]);
const kat = poseidon([1n, 2n]).toString();
if (kat !== '7853200120776062878684798364095072458815029376092732009249414926327459813530') throw new Error('KAT ' + kat);
for (const p of pairs.slice(0, 50)) poseidon(p);  // warm (JIT)
const t0 = process.hrtime.bigint();
let n = 0, acc = 0n;
while (Number(process.hrtime.bigint() - t0) < 10e9) {
  for (const p of pairs) { acc = (acc + poseidon(p)) % P; n++; }
}
const s = Number(process.hrtime.bigint() - t0) / 1e9;
const out = {
  what: "reference test/poseidon.js poseidon() (PoseidonEx(1, inputs, 0): every round's Sigma / Mix intermediates) " +
        "over config 1's 1,003 pairs, repeated for ~10 s",
  value: +(n / s).toFixed(1), unit: "hashes/s", cores: 1, sample: n + " hashes in " + s.toFixed(2) + " s",
  node: process.version, cpu: os.cpus()[0].model,
  measured_on: "the build container (8 CPUs), not the GPU box: the reference does not travel there", check: acc.toString(16).slice(0, 16)
};
fs.writeFileSync(process.argv[3], JSON.stringify(out, null, 1) + '\n');
console.log(JSON.stringify(out));
