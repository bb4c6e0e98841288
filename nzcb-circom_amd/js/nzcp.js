'use strict';
// NZ COVID Pass -> nzcp circuit input (SURVEY.md §8f rank 3), the step before
// plonk.fullProve: the pass URI's COSE_Sign1 is rebuilt into the ToBeSigned bytes the
// circuit hashes and parses (`NZCPPubIdentity`, /root/reference/circuits/nzcptpl.circom:444-655),
// packed as the reference's tests build the input (test/nzcp.js:33-42, helpers/utils.js:2-89):
//   toBeSigned: maxLen*8 bits MSB-first per byte, zero past the length; toBeSignedLen;
//   data: 20 bytes after the EVM byte/bit rearrangement (reversed bytes, reversed bits).
// The expected public signals follow the tests' decode (test/nzcp.js:44-68): three
// 248-bit big-endian words of nullifierHash[0..32) | sha256(ToBeSigned) | exp | data.
// Formats: base32 (RFC 4648, no padding), CBOR (RFC 7049), COSE_Sign1 (RFC 8152, tag 18),
// CWT claims (RFC 8392; 4 = exp, 5 = nbf, "vc".credentialSubject).
const crypto = require('crypto');

const B32 = 'ABCDEFGHIJKLMNOPQRSTUVWXYZ234567';

function base32Decode(s) {
  const out = [];
  let acc = 0;
  let bits = 0;
  for (const ch of s) {
    const v = B32.indexOf(ch);
    if (v < 0) throw new Error('invalid base32 character');
    acc = ((acc << 5) | v) & 0xffff;
    bits += 5;
    if (bits >= 8) {
      bits -= 8;
      out.push((acc >> bits) & 0xff);
    }
  }
  return Buffer.from(out);
}

// minimal CBOR decoder: returns [value, nextOffset]; byte strings are Buffers,
// maps are Map objects (keys may be ints or strings), tags are {tag, value}
function cborDecode(buf, off) {
  const ib = buf[off++];
  if (ib === undefined) throw new Error('truncated CBOR');
  const major = ib >> 5;
  let info = ib & 31;
  let arg;
  if (info < 24) arg = info;
  else if (info === 24) arg = buf[off++];
  else if (info === 25) { arg = buf.readUInt16BE(off); off += 2; }
  else if (info === 26) { arg = buf.readUInt32BE(off); off += 4; }
  else if (info === 27) { arg = Number(buf.readBigUInt64BE(off)); off += 8; }
  else throw new Error('unsupported CBOR length encoding');
  switch (major) {
    case 0: return [arg, off];
    case 1: return [-1 - arg, off];
    case 2: return [buf.subarray(off, off + arg), off + arg];
    case 3: return [buf.subarray(off, off + arg).toString('utf8'), off + arg];
    case 4: {
      const a = [];
      for (let i = 0; i < arg; i++) { let v; [v, off] = cborDecode(buf, off); a.push(v); }
      return [a, off];
    }
    case 5: {
      const m = new Map();
      for (let i = 0; i < arg; i++) {
        let k; let v;
        [k, off] = cborDecode(buf, off);
        [v, off] = cborDecode(buf, off);
        m.set(k, v);
      }
      return [m, off];
    }
    case 6: { let v; [v, off] = cborDecode(buf, off); return [{ tag: arg, value: v }, off]; }
    default:
      if (info === 20) return [false, off];
      if (info === 21) return [true, off];
      if (info === 22) return [null, off];
      throw new Error('unsupported CBOR item');
  }
}

// CBOR byte-string header + bytes (definite length)
function cborBytes(b) {
  const n = b.length;
  let head;
  if (n < 24) head = [0x40 | n];
  else if (n < 256) head = [0x58, n];
  else if (n < 65536) head = [0x59, n >> 8, n & 0xff];
  else throw new Error('byte string too long');
  return Buffer.concat([Buffer.from(head), Buffer.from(b)]);
}

function decodePass(passURI) {
  const m = /^NZCP:\/(\d+)\/([A-Z2-7]+)$/.exec(passURI);
  if (!m) throw new Error('not an NZCP pass URI');
  const bytes = base32Decode(m[2]);
  const [cose] = cborDecode(bytes, 0);
  if (!cose || cose.tag !== 18 || !Array.isArray(cose.value) || cose.value.length !== 4) {
    throw new Error('not a COSE_Sign1 structure');
  }
  const [bodyProtected, , payload, signature] = cose.value;
  return { bodyProtected, payload, signature };
}

// COSE Sig_structure ["Signature1", body_protected, external_aad = h'', payload]
function toBeSigned(passURI) {
  const { bodyProtected, payload } = decodePass(passURI);
  return Buffer.concat([Buffer.from([0x84, 0x6a]), Buffer.from('Signature1', 'ascii'), cborBytes(bodyProtected),
    cborBytes(Buffer.alloc(0)), cborBytes(payload)]);
}

function claims(passURI) {
  const { payload } = decodePass(passURI);
  const [cwt] = cborDecode(payload, 0);
  const vc = cwt.get('vc');
  const subj = vc && vc.get('credentialSubject');
  return {
    exp: cwt.get(4),
    nbf: cwt.get(5),
    givenName: subj && subj.get('givenName'),
    familyName: subj && subj.get('familyName'),
    dob: subj && subj.get('dob'),
  };
}

function bitsMsbFirst(bytes) {
  const out = [];
  for (const b of bytes) for (let j = 7; j >= 0; j--) out.push((b >> j) & 1);
  return out;
}

// reversed byte order and reversed bit order within each byte
function evmRearrange(bytes) {
  const n = bytes.length;
  const out = Buffer.alloc(n);
  for (let i = 0; i < n; i++) {
    let b = bytes[n - 1 - i];
    let r = 0;
    for (let j = 0; j < 8; j++) { r = (r << 1) | (b & 1); b >>= 1; }
    out[i] = r;
  }
  return out;
}

const LIVE_TOBESIGNED_MAX = 351;
const EXAMPLE_TOBESIGNED_MAX = 314;

// circuit input object for NZCPPubIdentity (plonk.fullProve's `input`)
function circuitInput(passURI, data, maxLen) {
  maxLen = maxLen || LIVE_TOBESIGNED_MAX;
  const tbs = toBeSigned(passURI);
  if (tbs.length > maxLen) throw new Error(`ToBeSigned is ${tbs.length} bytes, circuit takes ${maxLen}`);
  const d = Buffer.from(data || Buffer.alloc(20));
  if (d.length !== 20) throw new Error('data must be 20 bytes');
  const fitted = Buffer.alloc(maxLen);
  tbs.copy(fitted);
  return { toBeSigned: bitsMsbFirst(fitted), toBeSignedLen: tbs.length, data: bitsMsbFirst(evmRearrange(d)) };
}

// the three public signals the circuit outputs, as decimal strings
function expectedPublicSignals(passURI, data) {
  const c = claims(passURI);
  const nullifier = Buffer.alloc(64);
  Buffer.from(`${c.givenName},${c.familyName},${c.dob}`, 'utf8').copy(nullifier);
  const nh = crypto.createHash('sha512').update(nullifier).digest();
  const th = crypto.createHash('sha256').update(toBeSigned(passURI)).digest();
  const exp = Buffer.alloc(4);
  exp.writeUInt32BE(c.exp >>> 0, 0);
  const d = Buffer.from(data || Buffer.alloc(20));
  const words = [
    nh.subarray(0, 31),
    Buffer.concat([nh.subarray(31, 32), th.subarray(0, 30)]),
    Buffer.concat([th.subarray(30, 32), exp, d, Buffer.alloc(5)]),
  ];
  return words.map((w) => BigInt('0x' + w.toString('hex')).toString());
}

module.exports = {
  base32Decode, cborDecode, decodePass, toBeSigned, claims, circuitInput, expectedPublicSignals,
  evmRearrange, LIVE_TOBESIGNED_MAX, EXAMPLE_TOBESIGNED_MAX,
};
