'use strict';
// snarkjs-compatible PLONK API on the MI355X prover (SURVEY.md §8b).
//
// Drop-in for the two calls the reference's callers make into snarkjs 0.4.12
// (/root/reference/package.json:18; the dapp and the `snarkjs plonk prove|fullprove`
// CLI, README.md:50-53):
//   plonk.prove(zkeyFileName, witnessFileName, logger)       -> Promise<{proof, publicSignals}>
//   plonk.fullProve(input, wasmFile, zkeyFileName, logger)   -> Promise<{proof, publicSignals}>
// File arguments accept a path, a Buffer/Uint8Array, or {type: "mem", data}.
// Blinding scalars are drawn like snarkjs's Fr.random() unless options.blinding
// (11 x 32-byte LE Buffer) is given -- fixed blinding makes proofs bit-reproducible.
const fs = require('fs');
const path = require('path');
const crypto = require('crypto');

// proof streams need more than HIP's default 4 hardware queues per process (kernels of
// independent streams sharing a queue serialise); read when HIP initialises
if ((process.env.GPU_MAX_HW_QUEUES || '4') === '4') process.env.GPU_MAX_HW_QUEUES = '24';
const addon = require(path.join(__dirname, 'build', 'nzcb.node'));

const R = BigInt('21888242871839275222246405745257275088548364400416034343698204186575808495617');
const BLINDING_BYTES = 11 * 32;

// File arguments: a path, {type: "mem", data}, or a Buffer / Uint8Array (used in place,
// not copied)
function readBin(x) {
  if (typeof x === 'string') return fs.readFileSync(x);
  if (x && x.type === 'mem') return Array.isArray(x.data) ? Buffer.from(x.data) : readBin(x.data);
  if (Buffer.isBuffer(x)) return x;
  if (x instanceof Uint8Array) return Buffer.from(x.buffer, x.byteOffset, x.byteLength);
  throw new Error('expected a file name, a buffer or {type: "mem", data}');
}

function randomBlinding() {
  const out = Buffer.alloc(BLINDING_BYTES);
  const mask = (BigInt(1) << BigInt(254)) - BigInt(1);
  for (let i = 0; i < 11; i++) {
    let v;
    do {
      v = BigInt('0x' + crypto.randomBytes(32).toString('hex')) & mask;
    } while (v >= R);
    for (let j = 0; j < 32; j++) {
      out[32 * i + j] = Number(v & BigInt(255));
      v >>= BigInt(8);
    }
  }
  return out;
}

// One HBM-resident context per (zkey, device): the zkey is uploaded once. A file name is
// memory-mapped by the library (nzcb_ctx_create_file), so zkeys of nzcp_live size
// (~3.9 GB, beyond a Node Buffer) work; buffers are keyed by content. A context has
// `lanes` proof lanes: concurrent prove / fullProve promises on it run on different lanes at
// the same time. options.lanes (or NZCB_LANES) asks for an exact count; by default the
// context takes up to 5 (bench.py's measured best) as far as the device's free HBM allows
// (~6.5 GB per extra lane at n = 2^21): a lane count that does not fit is rolled back by
// the library and the next smaller one is tried.
const DEFAULT_LANES = 5;
const ENV_LANES = process.env.NZCB_LANES ? Number(process.env.NZCB_LANES) : 0;
const contexts = new Map();
// Buffer -> {hash, probe}: the content hash is computed once per Buffer; a cheap probe
// (length, head and tail bytes) is checked on every lookup, so a caller that reuses one
// Buffer for another zkey or program gets it hashed again rather than the old context.
// Mutating a Buffer in the middle is not detected: pass a fresh Buffer for new contents.
const bufHashes = new WeakMap();
function probeOf(buf) {
  const k = Math.min(buf.length, 4096);
  return crypto.createHash('sha1').update(buf.subarray(0, k)).update(buf.subarray(buf.length - k))
    .update(String(buf.length)).digest('hex');
}
function contentHash(buf) {
  const probe = probeOf(buf);
  const e = bufHashes.get(buf);
  if (e && e.probe === probe) return e.hash;
  const hash = crypto.createHash('sha256').update(buf).digest('hex');
  bufHashes.set(buf, { hash, probe });
  return hash;
}
function setLanesFitting(ctx, want) {
  for (let l = want; ; l--) {
    try {
      return addon.setLanes(ctx, l);
    } catch (e) {
      if (l <= 1) throw e;
    }
  }
}
function contextFor(zkey, device, lanes) {
  let key;
  if (typeof zkey === 'string') {
    const st = fs.statSync(zkey);
    key = `file:${path.resolve(zkey)}:${st.size}:${st.mtimeMs}:${device}`;
  } else {
    key = contentHash(readBin(zkey)) + ':' + device;
  }
  lanes = lanes || ENV_LANES;
  let c = contexts.get(key);
  if (!c) {
    const ctx = typeof zkey === 'string' ? addon.createContextFile(zkey, device) : addon.createContext(readBin(zkey), device);
    try {
      c = { ctx, lanes: lanes ? addon.setLanes(ctx, lanes) : setLanesFitting(ctx, DEFAULT_LANES) };
    } catch (e) {
      addon.releaseContext(ctx);  // its HBM now, not at garbage collection
      throw e;
    }
    contexts.set(key, c);
  } else if (lanes && lanes !== c.lanes) {
    // a change of lane count waits for the proofs in flight (it rebuilds the lane pool)
    addon.setLanes(c.ctx, lanes);
    c.lanes = lanes;
  }
  return c.ctx;
}

function loggerFn(logger) {
  if (!logger) return null;
  if (typeof logger === 'function') return logger;
  if (typeof logger.debug === 'function') return (m) => logger.debug(m);
  return null;
}

async function prove(zkeyFileName, witnessFileName, logger, options) {
  options = options || {};
  const wtns = readBin(witnessFileName);
  const ctx = contextFor(zkeyFileName, options.device || 0, options.lanes);
  const res = await addon.prove(ctx, wtns, blindingFor(options), loggerFn(logger));
  return { proof: JSON.parse(res.proof), publicSignals: JSON.parse(res.publicSignals) };
}

function blindingFor(options) {
  const blinding = options.blinding ? Buffer.from(options.blinding) : randomBlinding();
  if (blinding.length !== BLINDING_BYTES) throw new Error('blinding must be 11 x 32 bytes');
  return blinding;
}

// ---------------------------------------------------------------------------
// Witness calculation from a circom 2.0.x witness .wasm (circom_runtime 0.1.17
// WitnessCalculatorBuilder / calculateWTNSBin interface, SURVEY.md §2 [EXT]).
// Parity unpinned: no circom artefact exists offline to test against.
// ---------------------------------------------------------------------------
function fnvHash(str) {
  const M = BigInt(2) ** BigInt(64);
  let h = BigInt('0xCBF29CE484222325');
  for (let i = 0; i < str.length; i++) {
    h ^= BigInt(str.charCodeAt(i));
    h = (h * BigInt('0x100000001B3')) % M;
  }
  return h.toString(16).padStart(16, '0');
}

function flatArray(a) {
  const res = [];
  (function fill(x) {
    if (Array.isArray(x)) x.forEach(fill);
    else res.push(x);
  })(a);
  return res;
}

async function wtnsCalculate(input, wasmFile) {
  const code = Buffer.isBuffer(wasmFile) ? wasmFile : readBin(wasmFile);
  let instance;
  let errStr = '';
  const getMessage = () => {
    let msg = '';
    let c = instance.exports.getMessageChar();
    while (c !== 0) {
      msg += String.fromCharCode(c);
      c = instance.exports.getMessageChar();
    }
    return msg;
  };
  const errors = ['', 'Signal not found.', 'Too many signals set.', 'Signal already set.', 'Assert Failed.',
    'Not enough memory.', 'Input signal array access exceeds the size.'];
  const mod = await WebAssembly.compile(code);
  instance = await WebAssembly.instantiate(mod, {
    runtime: {
      exceptionHandler: (c) => { throw new Error((errors[c] || 'Unknown error.') + '\n' + errStr); },
      printErrorMessage: () => { errStr += getMessage() + '\n'; },
      writeBufferMessage: () => { getMessage(); },
      showSharedRWMemory: () => {},
    },
  });
  const ex = instance.exports;
  const n32 = ex.getFieldNumLen32();
  ex.getRawPrime();
  let prime = BigInt(0);
  for (let j = n32 - 1; j >= 0; j--) prime = (prime << BigInt(32)) | BigInt(ex.readSharedRWMemory(j) >>> 0);
  const witnessSize = ex.getWitnessSize();
  ex.init(0);
  let counter = 0;
  for (const k of Object.keys(input)) {
    const h = fnvHash(k);
    const hMSB = parseInt(h.slice(0, 8), 16);
    const hLSB = parseInt(h.slice(8, 16), 16);
    const vals = flatArray(input[k]);
    const size = ex.getInputSignalSize(hMSB, hLSB);
    if (size < 0) throw new Error(`Signal ${k} not found\n`);
    if (vals.length < size) throw new Error(`Not enough values for input signal ${k}\n`);
    if (vals.length > size) throw new Error(`Too many values for input signal ${k}\n`);
    for (let i = 0; i < vals.length; i++) {
      let v = BigInt(vals[i]) % prime;
      if (v < BigInt(0)) v += prime;
      for (let j = 0; j < n32; j++) {
        ex.writeSharedRWMemory(j, Number(v & BigInt(0xffffffff)));
        v >>= BigInt(32);
      }
      ex.setInputSignal(hMSB, hLSB, i);
      counter++;
    }
  }
  if (ex.getInputSize && counter < ex.getInputSize()) {
    throw new Error(`Not all inputs have been set. Only ${counter} out of ${ex.getInputSize()}`);
  }
  const n8 = n32 * 4;
  const out = Buffer.alloc(12 + 12 + 4 + n8 + 4 + 12 + witnessSize * n8);
  let o = 0;
  out.write('wtns', 0, 'latin1'); o = 4;
  out.writeUInt32LE(2, o); o += 4;
  out.writeUInt32LE(2, o); o += 4;
  out.writeUInt32LE(1, o); o += 4;
  out.writeUInt32LE(8 + n8, o); out.writeUInt32LE(0, o + 4); o += 8;
  out.writeUInt32LE(n8, o); o += 4;
  ex.getRawPrime();
  for (let j = 0; j < n32; j++) { out.writeUInt32LE(ex.readSharedRWMemory(j) >>> 0, o); o += 4; }
  out.writeUInt32LE(witnessSize, o); o += 4;
  out.writeUInt32LE(2, o); o += 4;
  const s2 = witnessSize * n8;
  out.writeUInt32LE(s2 % 0x100000000, o); out.writeUInt32LE(Math.floor(s2 / 0x100000000), o + 4); o += 8;
  for (let i = 0; i < witnessSize; i++) {
    ex.getWitness(i);
    for (let j = 0; j < n32; j++) { out.writeUInt32LE(ex.readSharedRWMemory(j) >>> 0, o); o += 4; }
  }
  return out;
}

// ---------------------------------------------------------------------------
// Witness calculation on the GPU from a witness program (nzcb/circuit.py write_program:
// nzcp_live = NZCPPubIdentity(1, 351, 0, 4, 2, 4) compiled by nzcb/nzcpgen.py), the
// MI355X replacement of the circom wasm for circuits this build compiles. The program
// carries the main's input names and sizes; inputs are mapped by name, as circom does.
// ---------------------------------------------------------------------------
function programInputs(prog) {
  const u32 = (o) => prog.readUInt32LE(o);
  const nc = u32(24), nt = u32(28), no = u32(32), nlev = u32(36);
  let o = 40 + nc * 32 + nt * 8 + no * 32 + (2 * nlev + 1) * 4;
  const n = u32(o); o += 4;
  const names = [];
  for (let i = 0; i < n; i++) {
    const len = u32(o); o += 4;
    const name = prog.toString('utf8', o, o + len); o += len;
    names.push([name, u32(o)]); o += 4;
  }
  // a remapped program (wtns.remapProgram) writes witnesses of its wire map's length
  const mapped = o + 8 <= prog.length && prog.toString('latin1', o, o + 4) === 'wmap';
  return { nWires: mapped ? u32(o + 4) : u32(8), names };
}

// nzcb_wprog_remap: a witness program re-indexed to the wire order of another .sym (e.g.
// circom's nzcp_live.sym, whose zkey expects circom's order), matching signals by name
// against the program's own .sym. Arguments: Buffers or file names.
function remapProgram(program, ownSym, targetSym) {
  return addon.remapWitnessProgram(readBin(program), readBin(ownSym), readBin(targetSym));
}

// fullProve's program argument: a path is read again only when its size or mtime changes (a
// server passes the same path on every call)
const programFiles = new Map();
function readProgram(x) {
  if (typeof x !== 'string') return readBin(x);
  const st = fs.statSync(x);
  const f = programFiles.get(x);
  if (f && f.size === st.size && f.mtimeMs === st.mtimeMs) return f.buf;
  const buf = fs.readFileSync(x);
  programFiles.set(x, { size: st.size, mtimeMs: st.mtimeMs, buf });
  return buf;
}

// loaded programs by content hash; a Buffer seen before skips the hash (a program of
// nzcp_live's size takes tens of ms to hash: per call, that was the Node path's bottleneck)
const programs = new Map();
const programsByBuf = new WeakMap();
function programFor(progBuf, device) {
  let byDev = programsByBuf.get(progBuf);
  const probe = probeOf(progBuf);
  if (byDev && byDev.probe !== probe) byDev = null;  // the Buffer now holds other contents
  if (byDev && byDev.has(device)) return byDev.get(device);
  const key = contentHash(progBuf) + ':' + device;
  let p = programs.get(key);
  if (!p) {
    p = { handle: addon.createWitnessProgram(progBuf, device), meta: programInputs(progBuf) };
    programs.set(key, p);
  }
  if (!byDev) {
    programsByBuf.set(progBuf, (byDev = new Map()));
    byDev.probe = probe;
  }
  byDev.set(device, p);
  return p;
}

// one signal value -> 32-byte LE at buf[off] (buf zero-filled): small non-negative numbers
// directly, everything else reduced mod r and written as four 64-bit words
const M64 = (BigInt(1) << BigInt(64)) - BigInt(1);
const B64 = BigInt(64);
function putSignal(buf, off, x) {
  if (typeof x === 'number' && Number.isSafeInteger(x) && x >= 0) {
    buf.writeUIntLE(x % 0x1000000000000, off, 6);
    if (x >= 0x1000000000000) buf.writeUInt16LE(Math.floor(x / 0x1000000000000), off + 6);
    return;
  }
  let v = BigInt(x) % R;
  if (v < BigInt(0)) v += R;
  for (let j = 0; j < 4; j++) { buf.writeBigUInt64LE(v & M64, off + 8 * j); v >>= B64; }
}

// the main's input object -> n_inputs x 32-byte LE values, by the program's input names
function programInputBuffer(input, meta) {
  const vals = [];
  for (const [name, size] of meta.names) {
    if (!(name in input)) throw new Error(`Signal ${name} not found\n`);
    const flat = flatArray(input[name]);
    if (flat.length < size) throw new Error(`Not enough values for input signal ${name}\n`);
    if (flat.length > size) throw new Error(`Too many values for input signal ${name}\n`);
    vals.push(...flat);
  }
  for (const k of Object.keys(input)) {
    if (!meta.names.some(([n]) => n === k)) throw new Error(`Signal ${k} not found\n`);
  }
  const buf = Buffer.alloc(32 * vals.length);
  vals.forEach((x, i) => putSignal(buf, 32 * i, x));
  return buf;
}

async function wtnsCalculateGpu(input, progBuf, device) {
  const { handle, meta } = programFor(progBuf, device);
  const buf = programInputBuffer(input, meta);
  const wit = await addon.calculateWitness(handle, buf);
  const hdr = Buffer.alloc(12 + 12 + 4 + 32 + 4 + 12);
  let o = 0;
  hdr.write('wtns', 0, 'latin1'); o = 4;
  hdr.writeUInt32LE(2, o); o += 4;
  hdr.writeUInt32LE(2, o); o += 4;
  hdr.writeUInt32LE(1, o); o += 4;
  hdr.writeUInt32LE(40, o); hdr.writeUInt32LE(0, o + 4); o += 8;
  hdr.writeUInt32LE(32, o); o += 4;
  let r = R;
  for (let j = 0; j < 32; j++) { hdr[o + j] = Number(r & BigInt(255)); r >>= BigInt(8); }
  o += 32;
  hdr.writeUInt32LE(meta.nWires, o); o += 4;
  hdr.writeUInt32LE(2, o); o += 4;
  hdr.writeUInt32LE(wit.length % 0x100000000, o); hdr.writeUInt32LE(Math.floor(wit.length / 0x100000000), o + 4);
  return Buffer.concat([hdr, wit]);
}

// wasmFile: a circom 2.0.x witness .wasm (run on the host CPU, as snarkjs does) or a
// witness program ("nzwp", run on the GPU). With a witness program the witness never
// leaves HBM: the program writes it into a device buffer that the proof reads
// (addon.fullProveDevice); only the input signals go up and the proof comes back.
async function fullProve(input, wasmFile, zkeyFileName, logger, options) {
  options = options || {};
  const code = readProgram(wasmFile);
  const device = options.device || 0;
  if (code.slice(0, 4).toString('latin1') === 'nzwp') {
    const { handle, meta } = programFor(code, device);
    const ctx = contextFor(zkeyFileName, device, options.lanes);
    const res = await addon.fullProveDevice(ctx, handle, programInputBuffer(input, meta), blindingFor(options),
      loggerFn(logger));
    return { proof: JSON.parse(res.proof), publicSignals: JSON.parse(res.publicSignals) };
  }
  const wtns = await wtnsCalculate(input, code);
  return prove(zkeyFileName, { type: 'mem', data: wtns }, logger, options);
}

// ---------------------------------------------------------------------------
// Verification key, verifier, Solidity calldata (SURVEY.md §8f ranks 1 and 4):
// snarkjs zKey.exportVerificationKey / plonk.verify / plonk.exportSolidityCallData.
// ---------------------------------------------------------------------------
const PROOF_POINTS = ['A', 'B', 'C', 'Z', 'T1', 'T2', 'T3', 'Wxi', 'Wxiw'];
const PROOF_EVALS = ['eval_a', 'eval_b', 'eval_c', 'eval_s1', 'eval_s2', 'eval_zw', 'eval_r'];
const VK_POINTS = ['Qm', 'Ql', 'Qr', 'Qo', 'Qc', 'S1', 'S2', 'S3'];

function le32(x) {
  let v = BigInt(x);
  const out = Buffer.alloc(32);
  for (let i = 0; i < 32; i++) { out[i] = Number(v & BigInt(255)); v >>= BigInt(8); }
  return out;
}
function g1Buf(p) { return String(p[2]) === '0' ? Buffer.alloc(64) : Buffer.concat([le32(p[0]), le32(p[1])]); }
function proofBuf(proof) {
  return Buffer.concat(PROOF_POINTS.map((k) => g1Buf(proof[k])).concat(PROOF_EVALS.map((k) => le32(proof[k]))));
}
function pubBuf(pub) { return Buffer.concat(pub.map(le32).concat([Buffer.alloc(0)])); }
function vkBuf(vk) {
  const head = Buffer.alloc(8);
  head.writeUInt32LE(Number(vk.nPublic), 0);
  head.writeUInt32LE(Number(vk.power), 4);
  const x2 = vk.X_2;
  return Buffer.concat([head, le32(vk.k1), le32(vk.k2)].concat(VK_POINTS.map((k) => g1Buf(vk[k])))
    .concat([le32(x2[0][0]), le32(x2[0][1]), le32(x2[1][0]), le32(x2[1][1]), le32(vk.w)]));
}

// snarkjs plonk.setup(r1csName, ptauName, zkeyName, logger) (snarkjs 0.4.12
// plonk_setup.js, run at /root/reference/Makefile:55,60): writes the PLONK zkey.
// Names may also be {type: "mem", data} objects; a {type: "mem"} zkeyName receives
// the bytes in .data.
async function setup(r1csName, ptauName, zkeyName, logger, options) {
  options = options || {};
  const log = loggerFn(logger);
  const zkey = addon.plonkSetup(readBin(r1csName), readBin(ptauName), options.device || 0);
  if (zkeyName && typeof zkeyName === 'object') zkeyName.data = new Uint8Array(zkey);
  else fs.writeFileSync(zkeyName, zkey);
  if (log) log(`Plonk setup: zkey of ${zkey.length} bytes`);
  return 0;
}

// binary verification key of a zkey: a file name is memory-mapped by the library
// (nzcb_vk_from_zkey_file), so nzcp_live's ~3.9 GB zkey is never read into a Buffer
// (fs.readFileSync refuses files past 2 GiB)
function vkOf(zkey) {
  return typeof zkey === 'string' ? addon.vkFromZkeyFile(zkey) : addon.vkFromZkey(readBin(zkey));
}

async function exportVerificationKey(zkeyFileName) {
  return JSON.parse(addon.vkToJson(vkOf(zkeyFileName)));
}

// snarkjs zKey.exportSolidityVerifier(zkeyName, templates, logger) (`zkey export
// solidityverifier`, /root/reference/Makefile:57,62): the verifier contract's source.
// The snarkjs templates argument is not used (the contract is rendered by the library);
// options.name sets the contract name (the reference's deploy-script.js asks for "Verifier").
async function exportSolidityVerifier(zkeyFileName, templates, logger, options) {
  options = options || {};
  const tp = options.transcriptPublic === undefined ? true : !!options.transcriptPublic;
  const src = addon.vkToSolidity(vkOf(zkeyFileName), options.name || 'PlonkVerifier', tp);
  const log = loggerFn(logger);
  if (log) log(`Solidity verifier: ${src.length} bytes`);
  return src;
}

async function verify(vkVerifier, publicSignals, proof, logger, options) {
  options = options || {};
  const tp = options.transcriptPublic === undefined ? true : !!options.transcriptPublic;
  const ok = addon.verify(vkBuf(vkVerifier), proofBuf(proof), pubBuf(publicSignals), tp);
  const log = loggerFn(logger);
  if (log) log(ok ? 'OK!' : 'Invalid proof');
  return ok;
}

async function exportSolidityCallData(proof, publicSignals) {
  return addon.calldata(proofBuf(proof), pubBuf(publicSignals));
}

// nzcp witness on the GPU (include/nzcb.h nzcb_nzcp_witness): the NZCPPubIdentity
// public signals and semantic signals of one or more circuit inputs (the object
// plonk.fullProve takes, test/nzcp.js:41). Throws like calculateWitness when a pass
// fails one of the circuit's constraints.
const NZCP_PARAMS = { live: [1, 351, 0, 4], example: [0, 314, 0, 4] };
const NZCP_STATUS = ['ok', 'toBeSigned bit check', 'toBeSignedLen > MaxToBeSignedBytes',
  'LessThan operands out of range', 'QuinSelector index out of range', 'CBOR type is not a map',
  'CBOR map length > 23', 'CBOR type is not a string', 'negative toBeSignedLen (unpinned)'];
const NZCP_RECORD_BYTES = 288;

function fieldLE(v) {
  let x = BigInt(v) % R;
  if (x < BigInt(0)) x += R;
  return le32(x.toString());
}

function nzcpWitness(inputs, options) {
  options = options || {};
  const list = Array.isArray(inputs) ? inputs : [inputs];
  const params = options.params || NZCP_PARAMS[options.circuit || 'live'];
  const bufs = [];
  for (const inp of list) {
    if (inp.toBeSigned.length !== 8 * params[1] || inp.data.length !== 160) {
      throw new Error(`nzcp input: toBeSigned must have ${8 * params[1]} bits and data 160`);
    }
    for (const b of inp.toBeSigned) bufs.push(fieldLE(b));
    bufs.push(fieldLE(inp.toBeSignedLen));
    for (const b of inp.data) bufs.push(fieldLE(b));
  }
  const raw = addon.nzcpWitness(Buffer.concat(bufs), list.length, params, options.device || 0);
  const out = [];
  for (let i = 0; i < list.length; i++) {
    const r = raw.subarray(i * NZCP_RECORD_BYTES, (i + 1) * NZCP_RECORD_BYTES);
    const status = r.readInt32LE(0);
    if (status !== 0) {
      throw new Error(`Assert Failed (nzcp pass ${i}): ${NZCP_STATUS[status] || status} (detail ${r.readInt32LE(4)})`);
    }
    const nullifier = r.subarray(128, 192);
    out.push({
      publicSignals: [0, 1, 2].map((k) => BigInt('0x' + Buffer.from(r.subarray(192 + 32 * k, 224 + 32 * k))
        .reverse().toString('hex')).toString()),
      exp: r.readUInt32LE(8),
      vcPos: r.readInt32LE(12),
      nullifier: nullifier.subarray(0, Math.max(0, Math.min(64, r.readInt32LE(28)))).toString('latin1'),
      toBeSignedHash: r.subarray(32, 64).toString('hex'),
      nullifierHash: r.subarray(64, 128).toString('hex'),
    });
  }
  return Array.isArray(inputs) ? out : out[0];
}

module.exports = {
  plonk: { setup, prove, fullProve, verify, exportSolidityCallData },
  zKey: { exportVerificationKey, exportSolidityVerifier },
  nzcp: Object.assign({}, require('./nzcp.js'), { witness: nzcpWitness }),
  wtns: { calculate: wtnsCalculate, remapProgram },
  version: addon.version,
  deviceCount: addon.deviceCount,
  _addon: addon,
  _programInputBuffer: programInputBuffer,  // tests: the input signals' 32-byte encoding
};
