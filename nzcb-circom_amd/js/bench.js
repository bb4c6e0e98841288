'use strict';
// Node.js throughput of the drop-in boundary (VERDICT r3 item 3): N concurrent
// plonk.fullProve calls of nzcp_live through the snarkjs-shaped API, as a dapp backend would
// make them (the reference's caller, /root/reference/README.md:50-53), against bench.py's
// proofs/s on the same box. Driven by tools/node_bench.py, which writes the zkey, the witness
// program and the passes' input objects (bench.py's passes: pass_data(i)).
//   node bench.js <zkey> <program.nzwp> <inputs.json> [concurrency] [lanes] [warmup]
const fs = require('fs');
const crypto = require('crypto');
const m = require('./');

const R = BigInt('21888242871839275222246405745257275088548364400416034343698204186575808495617');

function blinding(i) {  // distinct deterministic blinding per proof (bench.py blinding_for)
  const out = Buffer.alloc(11 * 32);
  for (let k = 0; k < 11; k++) {
    const h = crypto.createHash('sha256').update(Buffer.concat([Buffer.from('nzcb-bench'),
      Buffer.from(Uint32Array.of(i).buffer), Buffer.from([k])])).digest();
    let v = BigInt('0x' + h.toString('hex')) % R;
    for (let j = 0; j < 32; j++) { out[32 * k + j] = Number(v & BigInt(255)); v >>= BigInt(8); }
  }
  return out;
}

(async () => {
  const [zkey, prog, inputsPath] = process.argv.slice(2, 5);
  const conc = Number(process.argv[5] || 10);
  const lanes = Number(process.argv[6] || 5);
  const warmup = Number(process.argv[7] || 5);
  const inputs = JSON.parse(fs.readFileSync(inputsPath));
  const program = fs.readFileSync(prog);
  const vk = await m.zKey.exportVerificationKey(zkey);
  // `conc` requests in flight at a time (a server's concurrent callers)
  const run = async (items) => {
    const out = new Array(items.length);
    let next = 0;
    const worker = async () => {
      for (;;) {
        const i = next++;
        if (i >= items.length) return;
        out[i] = await m.plonk.fullProve(items[i].input, program, zkey, null, { blinding: blinding(items[i].id), lanes });
      }
    };
    await Promise.all([...Array(Math.min(conc, items.length)).keys()].map(worker));
    return out;
  };
  await run(inputs.slice(0, warmup).map((input, id) => ({ input, id: 999000 + id })));
  const t0 = process.hrtime.bigint();
  const res = await run(inputs.map((input, id) => ({ input, id })));
  const dt = Number(process.hrtime.bigint() - t0) / 1e9;
  const ok = await m.plonk.verify(vk, res[0].publicSignals, res[0].proof) &&
             await m.plonk.verify(vk, res[res.length - 1].publicSignals, res[res.length - 1].proof);
  const distinct = new Set(res.map((r) => JSON.stringify(r.proof))).size;
  console.log(JSON.stringify({
    metric: 'node_fullprove_proofs_per_s', value: res.length / dt, proofs: res.length, seconds: dt,
    concurrency: conc, lanes, verified: ok, distinct_proofs: distinct,
    publicSignals0: res[0].publicSignals,
  }));
  if (!ok || distinct !== res.length) process.exit(1);
})().catch((e) => { console.error(e); process.exit(1); });
