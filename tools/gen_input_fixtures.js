// Runs the REFERENCE's own input-preparation functions (test/process_passport.js) on raw passport
// data in this container and writes their outputs as fixtures. The reference never travels to the
// GPU box; only the JSON this writes is committed (tests/golden/process_passport_vectors.json).
//   node tools/gen_input_fixtures.js /root/reference/test cases.json out.json
//
// process_passport.js as a whole does not parse on this Node 12 (optional chaining at :330) and
// its ./asn1.js dependency neither, so the functions are cut out of its source text by name and
// evaluated in a sandbox with the same free variables they use at module scope:
//   padding            :11-91     computeHash        :93-111    bigintToArray      :113-123
//   bigintToArrayString :125-135  getChunkedParams   :592-626   getFakeIdenData    :628-657
//   reHex              :6         poseidon           test/poseidon.js:134-137 (require)
// The glue that turns padding()'s hex into the bit arrays of the input JSON is restated from
// processPassport (:701-757: BigInt(...).toString(2).split(""), then left zero-fill to a multiple
// of the block length), as is the JSON assembly of writeToJson (:659-672).
"use strict";
const fs = require("fs");
const path = require("path");
const vm = require("vm");
const crypto = require("crypto");

const refDir = path.resolve(process.argv[2]);
const cases = JSON.parse(fs.readFileSync(process.argv[3], "utf8"));
const outPath = process.argv[4];
const src = fs.readFileSync(path.join(refDir, "process_passport.js"), "utf8");

function cut(name) {
  const at = src.indexOf("function " + name + "(");
  if (at < 0) throw new Error("function " + name + " not found");
  let i = src.indexOf("{", src.indexOf(")", at)), depth = 0;
  for (let j = i; j < src.length; j++) {
    if (src[j] === "{") depth++;
    else if (src[j] === "}" && --depth === 0) return { text: src.slice(at, j + 1), line: src.slice(0, at).split("\n").length };
  }
  throw new Error("unbalanced " + name);
}
const reHexLine = src.split("\n").find((l) => l.startsWith("const reHex"));
const names = ["padding", "computeHash", "bigintToArray", "bigintToArrayString", "getChunkedParams", "getFakeIdenData"];
const pieces = names.map(cut);
const ctx = vm.createContext({ BigInt, Buffer, Uint8Array, Array, Math, Error, parseInt,
                               createHash: crypto.createHash,
                               poseidon: require(path.join(refDir, "poseidon.js")).poseidon });
vm.runInContext(reHexLine + "\n" + pieces.map((p) => p.text).join("\n") + "\nthis.F = {" + names.join(",") + "};", ctx);
const F = ctx.F;

// processPassport :701-757
function paddedBits(hex, blockBits) {
  let bits = BigInt("0x" + F.padding(hex, blockBits)).toString(2).split("");
  if (bits.length % blockBits !== 0) bits = Array(blockBits - (bits.length % blockBits)).fill("0").concat(bits);
  return bits.join("");
}

const out = { source: "reference test/process_passport.js (functions at lines " +
                      pieces.map((p, k) => names[k] + ":" + p.line).join(", ") + ") run on node " + process.version,
              cases: [] };
for (const c of cases) {
  const r = { name: c.name, sig_type: c.sig_type, index: c.index, seed: c.seed };
  if (c.padding) r.padding = c.padding.map(([hex, bb]) => ({ hex, block_bits: bb, padded: F.padding(hex, bb), bits: paddedBits(hex, bb) }));
  if (c.limbs) r.limbs = c.limbs.map(([n, k, x]) => ({ n, k, x, array: F.bigintToArray(n, k, BigInt(x)).map(String),
                                                        array_string: F.bigintToArrayString(n, k, BigInt(x)) }));
  if (c.hash) r.hash = c.hash.map(([len, hex]) => ({ len, hex, digest: Buffer.from(F.computeHash(len, Buffer.from(hex, "hex"))).toString("hex") }));
  if (c.passport) {
    const p = c.passport;
    const blk = p.hash_block_bits || 512, dblk = p.dg_block_bits || 512;
    const chunked = F.getChunkedParams(p.pk, p.sig);
    const [sk, root, branches] = F.getFakeIdenData(Uint8Array.from(Buffer.from(p.ec, "hex")), p.pk);
    r.passport = {
      raw: p,
      json: {  // writeToJson :659-672 of processPassport's arrays (bit arrays stored joined: "0101...")
        dg1: paddedBits(p.dg1, dblk),
        dg15: p.dg15.length ? paddedBits(p.dg15, dblk) : "",
        signedAttributes: paddedBits(p.sa, blk),
        encapsulatedContent: paddedBits(p.ec, blk),
        pubkey: chunked.pk_chunked,
        signature: chunked.sig_chunked,
        skIdentity: "0x" + sk,
        slaveMerkleRoot: "0x" + root,
        slaveMerkleInclusionBranches: new Array(80).fill("0"),
      },
      chunk_number: chunked.chunk_number, ec_field_size: chunked.ec_field_size, branches: branches.length,
    };
  }
  out.cases.push(r);
}
fs.writeFileSync(outPath, JSON.stringify(out));
console.log("wrote " + out.cases.length + " cases to " + outPath);
