// Tests of the JS host layer (run by tests/test_js.py).
//   node test_witness_calculator.js cpu                      addon loads, marshalling + error texts
//   node test_witness_calculator.js gpu IN.json OUT.wtns     Poseidon KAT, then the register
//                                                            witness of IN.json written as .wtns
"use strict";
const assert = require("assert");
const fs = require("fs");

const mode = process.argv[2] || "cpu";

function fakeCalc(groups) {
  // a WitnessCalculator shell for marshalling tests (no device needed)
  const { WitnessCalculator } = require("./witness_calculator.js");
  const o = Object.create(WitnessCalculator.prototype);
  o.inputs = new Map(groups.map((g) => [g.name, g]));
  o.nInputs = groups.reduce((a, g) => a + g.length, 0);
  return o;
}

async function cpu() {
  const wcmod = require("./witness_calculator.js");
  assert.ok(wcmod.version().startsWith("pzkwit"));
  // no GPU here: creating an instance must fail loudly (no CPU fallback)
  await assert.rejects(wcmod.builder({}), /no HIP device/);
  const c = fakeCalc([{ name: "a", offset: 0, length: 2 }, { name: "b", offset: 2, length: 1 }]);
  const buf = c.marshal({ a: [["1"], [2]], b: "0x10" });
  assert.strictEqual(buf[0], 1);
  assert.strictEqual(buf[32], 2);
  assert.strictEqual(buf[64], 16);
  const m1 = c.marshal({ a: ["-1", 0], b: 5n });  // negative values reduce mod p
  const pm1 = wcmod.PRIME - 1n;
  let x = 0n;
  for (let j = 31; j >= 0; j--) x = (x << 8n) | BigInt(m1[j]);
  assert.strictEqual(x, pm1);
  assert.throws(() => c.marshal({ a: [1, 2], b: 1, zz: 3 }), /Signal zz not found/);
  assert.throws(() => c.marshal({ a: [1], b: 1 }), /Not enough values for input signal a/);
  assert.throws(() => c.marshal({ a: [1, 2, 3], b: 1 }), /Too many values for input signal a/);
  assert.throws(() => c.marshal({ a: [1, 2] }), /Not all inputs have been set/);
  assert.ok(/Error in template RsaVerifyPkcs1v15 line: 48/.test(wcmod.statusMessage(8)));
  assert.ok(/Error in template verifyECDSABits line: 81/.test(wcmod.statusMessage(16)));
  assert.ok(/Error in template VerifyRsaPssSig line: 182/.test(wcmod.statusMessage(18)));
  assert.strictEqual(wcmod.CIRCUIT.SHA1, 3);
  console.log("js cpu ok");
}

async function gpu(inPath, outPath) {
  const { builder, CIRCUIT } = require("./witness_calculator.js");
  // Poseidon(2) KAT from the reference's test/poseidon.js (SURVEY.md §8c)
  const pc = await builder({ circuit: CIRCUIT.POSEIDON, sizeArg: 2 });
  const w = await pc.calculateWitness({ in: ["1", "2"] }, true);
  assert.strictEqual(w[0], 1n);
  assert.strictEqual(w[1], 7853200120776062878684798364095072458815029376092732009249414926327459813530n);
  const rc = await builder({ circuit: CIRCUIT.REGISTER });
  const input = JSON.parse(fs.readFileSync(inPath, "utf8"));
  const t0 = Date.now();
  const wtns = await rc.calculateWTNSBin(input, true);
  fs.writeFileSync(outPath, Buffer.from(wtns.buffer, wtns.byteOffset, wtns.length));
  // batch path: two copies of the same passport give identical .wtns
  const b = await rc.calculateWTNSBinBatch([input, input], true);
  assert.strictEqual(b.status.length, 2);
  assert.ok(Buffer.compare(Buffer.from(b.wtns[0]), Buffer.from(b.wtns[1])) === 0);
  assert.ok(Buffer.compare(Buffer.from(b.wtns[0]), Buffer.from(wtns)) === 0);
  // concurrent, unawaited calls on one instance (libuv pool threads): serialised inside the
  // library, each result equal to the serial one
  const conc = await Promise.all([rc.calculateWTNSBin(input, true), rc.calculateWTNSBinBatch([input, input], true),
                                  rc.calculateWTNSBin(input, true)]);
  for (const x of [conc[0], conc[1].wtns[0], conc[1].wtns[1], conc[2]])
    assert.ok(Buffer.compare(Buffer.from(x), Buffer.from(wtns)) === 0);
  console.log(`js gpu ok (witnessSize ${rc.witnessSize}, ${Date.now() - t0} ms)`);
}

(mode === "cpu" ? cpu() : gpu(process.argv[3], process.argv[4])).catch((e) => {
  console.error(e);
  process.exit(1);
});
