// Tests of the JS host layer (run by tests/test_js.py).
//   node test_witness_calculator.js cpu [PP.json ROWS.bin]   addon loads, marshalling + error texts; with
//        PP.json ({ params, passports: [{dg1, dg15, sod} base64], names }) the bulk preprocessor binding:
//        passportParse names and passportInputs rows == ROWS.bin (the C-ABI's rows, via Python)
//   node test_witness_calculator.js gpu IN.json OUT.wtns [EXTRA.json [OUTDIR]]
//        Poseidon KAT, then the register witness of IN.json written as .wtns; with EXTRA.json
//        ({ inputs: [3 passports' JSON], sym: ".sym text" }) concurrent calls on different passports, a
//        .sym-mapped instance, and the streamed forms: 64 witnesses in chunks of 16 checked against the serial
//        results with the process's resident memory bounded by two chunks, an async sink, a sink that stops the
//        stream, and (OUTDIR) writeWTNSFiles of [IN, 3 passports] as OUTDIR/w<i>.wtns
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
  if (ppPath) {
    const pp = JSON.parse(fs.readFileSync(ppPath, "utf8"));
    const b64 = (x) => (x ? Buffer.from(x, "base64") : null);
    const passports = pp.passports.map((p) => ({ dg1: b64(p.dg1), dg15: b64(p.dg15), sod: b64(p.sod) }));
    passports.forEach((p, i) => assert.strictEqual(wcmod.passportParse(p).name, pp.names[i]));
    assert.throws(() => wcmod.passportParse({ dg1: Buffer.from([0x61]), sod: Buffer.from([0x30, 0x80]) }),
                  /pzk_passport_parse/);
    const r = await wcmod.passportInputs(pp.params, passports, null, 2);
    const want = fs.readFileSync(rowsPath);
    assert.strictEqual(r.status.length, passports.length);
    assert.ok(Buffer.compare(r.rows, want) === 0, "passportInputs rows differ from the C-ABI's");
    assert.deepStrictEqual(Array.from(r.status), pp.status);
  }
  console.log("js cpu ok");
}

async function gpu(inPath, outPath, extraPath) {
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
  if (extraPath) {
    const extra = JSON.parse(fs.readFileSync(extraPath, "utf8"));
    const [a, b, c] = extra.inputs;
    // serial results of three different passports
    const ser = [];
    for (const x of [a, b, c]) ser.push(Buffer.from(await rc.calculateWTNSBin(x, true)));
    assert.ok(Buffer.compare(ser[0], ser[1]) !== 0 && Buffer.compare(ser[1], ser[2]) !== 0);
    // concurrent, unawaited calls on one instance (libuv pool threads), each on its own passports: serialised
    // inside the library; every result equals ITS passport's serial result (a cross-call buffer mix-up fails)
    const conc = await Promise.all([rc.calculateWTNSBin(a, true), rc.calculateWTNSBinBatch([b, c], true),
                                    rc.calculateWTNSBin(c, true), rc.calculateWTNSBinBatch([c, a], true),
                                    rc.calculateWTNSBin(b, true)]);
    const got = [[conc[0], 0], [conc[1].wtns[0], 1], [conc[1].wtns[1], 2], [conc[2], 2], [conc[3].wtns[0], 2],
                 [conc[3].wtns[1], 0], [conc[4], 1]];
    got.forEach(([x, k], i) => assert.ok(Buffer.compare(Buffer.from(x), ser[k]) === 0, `concurrent result ${i}`));
    // a .sym-mapped instance: element k of its witness = O0 signal inv[k] of the unmapped one
    const inv = [0];
    for (const ln of extra.sym.split("\n")) {
      if (!ln) continue;
      const [sig, wi] = ln.split(",").map(Number);
      if (wi >= 0 && (inv[wi] === undefined || sig < inv[wi])) inv[wi] = sig;
    }
    const mc = await builder({ circuit: CIRCUIT.REGISTER }, { sym: extra.sym });
    assert.strictEqual(mc.witnessSize, inv.length);
    const mw = Buffer.from(await mc.calculateWTNSBin(b, true));
    assert.strictEqual(mw.length, 76 + 32 * inv.length);
    assert.strictEqual(mw.readUInt32LE(60), inv.length);  // header witnessSize (after the prime)
    const o0 = ser[1];
    for (let k = 0; k < inv.length; k++)
      if (Buffer.compare(mw.subarray(76 + 32 * k, 108 + 32 * k), o0.subarray(76 + 32 * inv[k], 108 + 32 * inv[k])) !== 0)
        throw new Error(`mapped element ${k} (signal ${inv[k]}) differs`);
  }
  if (extraPath) {
    const extra = JSON.parse(fs.readFileSync(extraPath, "utf8"));
    const three = extra.inputs;
    const ser = [];
    for (const x of three) ser.push(Buffer.from(await rc.calculateWTNSBin(x, true)));
    const rowBytes = rc.witnessSize * 32, chunk = 16, n = 64;
    // streamed, 64 witnesses (the three passports tiled) in chunks of 16: every witness equals its passport's
    // serial .wtns, in order, and the resident set grows by about two chunks of rows (the library's pinned
    // slots), not by the 64 witnesses a batch call would hold
    const inputs64 = Array.from({ length: n }, (_, i) => three[i % 3]);
    global.gc && global.gc();
    const rss0 = process.memoryUsage().rss;
    let peak = rss0, next = 0;
    await rc.calculateWTNSBinStream(inputs64, (i, header, witness, st) => {
      assert.strictEqual(i, next++);
      assert.strictEqual(st, 0);
      assert.ok(Buffer.compare(Buffer.from(header), ser[i % 3].subarray(0, 76)) === 0, `header ${i}`);
      assert.ok(Buffer.compare(witness, ser[i % 3].subarray(76)) === 0, `streamed witness ${i}`);
      peak = Math.max(peak, process.memoryUsage().rss);
    }, true, chunk);
    assert.strictEqual(next, n);
    const grew = peak - rss0, bound = 2.5 * chunk * rowBytes + 512e6;
    assert.ok(grew < bound && grew < n * rowBytes, `resident set grew ${grew} B (bound ${bound})`);
    // an async sink: the library waits for each chunk's promise before reusing its pinned slot
    let seen = 0;
    await rc.calculateWTNSBinStream(inputs64.slice(0, 8), async (i, header, witness) => {
      await new Promise((r) => setTimeout(r, 1));
      assert.ok(Buffer.compare(witness, ser[i % 3].subarray(76)) === 0, `async sink ${i}`);
      seen++;
    }, true, 3);
    assert.strictEqual(seen, 8);
    // a throwing sink stops the stream and rejects with its own error
    await assert.rejects(rc.calculateWTNSBinStream(inputs64.slice(0, 6), (i) => {
      if (i === 3) throw new Error("stop at 3");
    }, true, 2), /stop at 3/);
    // a view kept past its callback is detached when the chunk is done (reads as empty, never as a recycled slot)
    const kept = [];
    await rc.calculateWTNSBinStream(inputs64.slice(0, 4), (i, header, witness) => { kept.push(witness); }, true, 2);
    assert.ok(kept.length === 4 && kept.every((w) => w.length === 0), `kept views: ${kept.map((w) => w.length)}`);
    // a call into the same calculator from inside onWitness rejects instead of deadlocking on the instance
    let reentrant = null;
    await rc.calculateWTNSBinStream(inputs64.slice(0, 2), async () => {
      try { await rc.calculateWTNSBin(three[0], true); } catch (e) { reentrant = e; }
    }, true, 2);
    assert.ok(reentrant && /streaming/.test(reentrant.message), `re-entrant call: ${reentrant}`);
    // a failing lane with sanityCheck rejects before any onWitness of its chunk runs
    const bad = JSON.parse(JSON.stringify(three[0]));
    bad.dg1[10] = bad.dg1[10] === "1" ? "0" : "1";  // dg1 hash != the EC field -> flow check (code 7)
    let called = 0;
    await assert.rejects(rc.calculateWTNSBinStream([three[1], bad], async () => { called++; }, true, 2),
                         /Assert Failed/);
    assert.strictEqual(called, 0);
    // the instance still works after a stopped stream
    const again = Buffer.from(await rc.calculateWTNSBin(three[0], true));
    assert.ok(Buffer.compare(again, ser[0]) === 0);
    if (outDir) {
      const path = require("path");
      const cnt = await rc.writeWTNSFiles([input].concat(three), (i) => path.join(outDir, `w${i}.wtns`), true, 2);
      assert.strictEqual(cnt, 4);
    }
    console.log(`js stream ok (64 witnesses, resident +${(grew / 1e9).toFixed(2)} GB for chunks of ${chunk})`);
  }
  console.log(`js gpu ok (witnessSize ${rc.witnessSize}, ${Date.now() - t0} ms)`);
}

const ppPath = mode === "cpu" ? process.argv[3] : null, rowsPath = process.argv[4], outDir = process.argv[6];
(mode === "cpu" ? cpu() : gpu(process.argv[3], process.argv[4], process.argv[5])).catch((e) => {
  console.error(e);
  process.exit(1);
});
