// Runs the REFERENCE's own processPassport (test/process_passport.js:674-816) over synthetic passport
// files ({dg1, dg15, sod}, base64; pzkwit/sodgen.py) in this container and collects what it writes:
// the RegisterIdentityBuilder parameters of the generated .circom (writeToCircom :573-588) and the
// input JSON (writeToJson :659-672). Only the collected JSON is committed (tests/golden/sod_vectors.json);
// the reference never travels to the GPU box.
//   node --harmony-optional-chaining --harmony-private-methods tools/gen_sod_fixtures.js \
//        /root/reference/test cases_dir out.json
// The two V8 flags let this Node 12 parse the reference's optional chaining (:330-370) and
// asn1.js's private class members. asn1.js's Hex decoder does not run under them, so every field is
// base64 (processPassport's other branch, Base64.unarmor). processPassport writes into
// test/circuits/generated and test/inputs/generated under the working directory: it runs in a
// scratch directory here.
"use strict";
const fs = require("fs");
const os = require("os");
const path = require("path");

const refDir = path.resolve(process.argv[2]);
const casesDir = path.resolve(process.argv[3]);
const outPath = path.resolve(process.argv[4]);
const { processPassport } = require(path.join(refDir, "process_passport.js"));

const work = fs.mkdtempSync(path.join(os.tmpdir(), "sodfix-"));
fs.mkdirSync(path.join(work, "test", "circuits", "generated"), { recursive: true });
fs.mkdirSync(path.join(work, "test", "inputs", "generated"), { recursive: true });
process.chdir(work);

const bits = (a) => (Array.isArray(a) ? a.join("") : a);
const out = { source: "reference test/process_passport.js processPassport run on node " + process.version, cases: [] };
for (const f of fs.readdirSync(casesDir).filter((x) => x.endsWith(".json")).sort()) {
  const name = processPassport(path.join(casesDir, f));
  const circom = fs.readFileSync(path.join(work, "test", "circuits", "generated", name + ".circom"), "utf8");
  const args = circom.slice(circom.indexOf("RegisterIdentityBuilder(") + 24, circom.lastIndexOf(")"))
    .split("\n").map((l) => l.replace(/\/\/.*$/, "").trim().replace(/,$/, "")).filter((l) => l.length);
  const j = JSON.parse(fs.readFileSync(path.join(work, "test", "inputs", "generated", name + ".json"), "utf8"));
  out.cases.push({
    file: f, name, circom_args: args,
    inputs: { dg1: bits(j.dg1), dg15: bits(j.dg15), signedAttributes: bits(j.signedAttributes),
              encapsulatedContent: bits(j.encapsulatedContent), pubkey: j.pubkey, signature: j.signature,
              skIdentity: j.skIdentity, slaveMerkleRoot: j.slaveMerkleRoot,
              branches: j.slaveMerkleInclusionBranches.length },
  });
}
fs.writeFileSync(outPath, JSON.stringify(out));
console.log("wrote " + out.cases.length + " cases to " + outPath);
