#!/usr/bin/env node
'use strict';
// `snarkjs plonk setup|prove|fullprove` equivalent on the MI355X prover (SURVEY.md §8b):
//   node cli.js plonk setup     <circuit.r1cs> <pot.ptau> <circuit.zkey>
//   node cli.js plonk prove     <circuit.zkey> <witness.wtns> <proof.json> <public.json>
//   node cli.js plonk fullprove <input.json> <circuit.wasm> <circuit.zkey> <proof.json> <public.json>
//   node cli.js plonk verify    <verification_key.json> <public.json> <proof.json>
//     (prints "OK!" and exits 0 for a valid proof, "Invalid proof" and exit code 1 otherwise,
//     as snarkjs's CLI verb; host only, no GPU)
// and `snarkjs zkey export verificationkey|solidityverifier|soliditycalldata` (Makefile:56-62):
//   node cli.js zkey export verificationkey <circuit.zkey> <verification_key.json>
//   node cli.js zkey export solidityverifier <circuit.zkey> <Verifier.sol> [contract name]
//   node cli.js zkey export soliditycalldata <public.json> <proof.json>
// Output JSON is written like snarkjs's CLI (stringifyBigInts, 1-space indent).
const fs = require('fs');
const nz = require('./index.js');

function usage() {
  console.error('usage: cli.js plonk setup <r1cs> <ptau> <zkey>\n' +
                '       cli.js plonk prove <zkey> <wtns> <proof.json> <public.json>\n' +
                '       cli.js plonk fullprove <input.json> <wasm> <zkey> <proof.json> <public.json>\n' +
                '       cli.js plonk verify <verification_key.json> <public.json> <proof.json>\n' +
                '       cli.js zkey export verificationkey <zkey> <verification_key.json>\n' +
                '       cli.js zkey export solidityverifier <zkey> <verifier.sol> [contract name]\n' +
                '       cli.js zkey export soliditycalldata <public.json> <proof.json>');
  process.exit(1);
}

async function zkeyExport(argv) {
  if (argv[1] !== 'export') usage();
  if (argv[2] === 'verificationkey' && argv.length === 5) {
    const vk = await nz.zKey.exportVerificationKey(argv[3]);
    fs.writeFileSync(argv[4], JSON.stringify(vk, null, 1), 'utf-8');
  } else if (argv[2] === 'solidityverifier' && (argv.length === 5 || argv.length === 6)) {
    const src = await nz.zKey.exportSolidityVerifier(argv[3], null, null, { name: argv[5] });
    fs.writeFileSync(argv[4], src, 'utf-8');
  } else if (argv[2] === 'soliditycalldata' && argv.length === 5) {
    const pub = JSON.parse(fs.readFileSync(argv[3], 'utf8'));
    const proof = JSON.parse(fs.readFileSync(argv[4], 'utf8'));
    console.log(await nz.plonk.exportSolidityCallData(proof, pub));
  } else {
    usage();
  }
}

async function main(argv) {
  if (argv[0] === 'zkey') return zkeyExport(argv);
  if (argv[0] !== 'plonk') usage();
  const logger = process.env.NZCB_VERBOSE ? { debug: (m) => console.error(m) } : null;
  let res, out;
  if (argv[1] === 'setup' && argv.length === 5) {
    await nz.plonk.setup(argv[2], argv[3], argv[4], logger);
    return;
  }
  if (argv[1] === 'verify' && argv.length === 5) {
    const vk = JSON.parse(fs.readFileSync(argv[2], 'utf8'));
    const pub = JSON.parse(fs.readFileSync(argv[3], 'utf8'));
    const proof = JSON.parse(fs.readFileSync(argv[4], 'utf8'));
    const ok = await nz.plonk.verify(vk, pub, proof, logger);
    console.log(ok ? 'OK!' : 'Invalid proof');
    process.exit(ok ? 0 : 1);
  }
  if (argv[1] === 'prove' && argv.length === 6) {
    res = await nz.plonk.prove(argv[2], argv[3], logger);
    out = argv.slice(4);
  } else if (argv[1] === 'fullprove' && argv.length === 7) {
    const input = JSON.parse(fs.readFileSync(argv[2], 'utf8'));
    res = await nz.plonk.fullProve(input, argv[3], argv[4], logger);
    out = argv.slice(5);
  } else {
    usage();
  }
  fs.writeFileSync(out[0], JSON.stringify(res.proof, null, 1), 'utf-8');
  fs.writeFileSync(out[1], JSON.stringify(res.publicSignals, null, 1), 'utf-8');
}

main(process.argv.slice(2)).then(() => process.exit(0), (e) => {
  console.error(e && e.message ? e.message : e);
  process.exit(1);
});
