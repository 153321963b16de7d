// fgv_msp.cpp -- the MSP cache miss on the engine side (fgv_msp_resolve*, include/fgv.h).
//
// The peer's MSP cache (msp/cache/cache.go:65-83) hands an identity it has not seen to the
// channel's MSP, which deserializes and validates the certificate (bccspmsp, MSP version 1.4.3):
//   mspimpl.go:398-422   deserializeIdentityInternal: pem.Decode, x509.ParseCertificate, bccsp
//                        KeyImport (Ed25519 fails)
//   identities.go:48-84  newIdentity: sanitizeCert, then Id = SHA-256 of the sanitized cert
//   mspimpl.go:892-938   sanitizeCert: chain to a root (x509 Verify at NotBefore + 1 s, exactly
//                        one chain; else DeserializeIdentity fails), re-marshal with a low-S
//                        signature
//   mspimplvalidate.go   validateIdentity: the chain, the signing CA's SubjectKeyIdentifier,
//                        validateIdentityOUsV142 (OU identifiers; NodeOUs: exactly one role OU)
//   mspimpl.go:607-680   ROLE principals: MEMBER = Validate; ADMIN = in admins or (valid and
//                        admin OU); CLIENT / PEER / ORDERER = valid and that OU
// The MSP model is built from the channel configuration's FabricMSPConfig: root and intermediate
// CAs (each a CA with a SubjectKeyIdentifier, chains by unique issuer names, verified on the GPU
// at build; parents of intermediates are internal nodes of the certification tree, mspimpl.go:
// 835-858), no CRLs, OU certificates that are CAs of the MSP.  The CA signatures of a batch of
// misses are verified on the GPU in one pass (the CA keys are pinned key-table slots) and the
// results registered like fgv_msp_register_identity.  Shapes outside the model stay
// unregistered (the batch stays FGV_EUNSUPPORTED: the reference decides).  The same rules as
// oracle/msp.py + oracle/x509.py, which the parity tests compare against.
#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <memory>
#include <set>
#include <unordered_set>

#include "fgv_channel.h"
#include "fgv_internal.h"
#include "fgv_x509.h"
#include "sha256_host.h"

using fgvb::Channel;
using fgvb::Ident;
using pbw::Span;

namespace {

// ---- FabricMSPConfig (msp/msp_config.pb.go) visitors
struct VOUIdent {  // FabricOUIdentifier {certificate 1, organizational_unit_identifier 2}
  Span cert, ou;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_BYTES : f == 2 ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    (f == 1 ? cert : ou) = s;
    return true;
  }
};
struct VNodeOUs {  // FabricNodeOUs {enable 1, client 2, peer 3, admin 4, orderer 5}
  bool enable = false;
  std::vector<Span> role[6];  // by field number
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : (f >= 2 && f <= 5) ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { enable = v != 0; }
  bool on_len(uint32_t f, Span s) {
    role[f].push_back(s);
    return true;
  }
};
struct VCryptoCfg {  // FabricCryptoConfig {signature_hash_family 1, identity_identifier_hash_function 2}
  Span fam, idhash;
  pbw::Kind kind(uint32_t f) { return (f == 1 || f == 2) ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    (f == 1 ? fam : idhash) = s;
    return true;
  }
};
struct VMspCfg {  // FabricMSPConfig {name 1, root_certs 2, intermediate_certs 3, admins 4,
                  // revocation_list 5, organizational_unit_identifiers 7, crypto_config 8,
                  // fabric_node_ous 11}
  Span name;
  std::vector<Span> roots, inters, admins, crls, ous, crypto, node;
  pbw::Kind kind(uint32_t f) {
    switch (f) {
      case 1: return pbw::K_STRING;
      case 2: case 3: case 4: case 5: return pbw::K_REP_BYTES;
      case 7: return pbw::K_REP_MSG;
      case 8: case 11: return pbw::K_MSG;
      default: return pbw::K_NONE;
    }
  }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    switch (f) {
      case 1: name = s; break;
      case 2: roots.push_back(s); break;
      case 3: inters.push_back(s); break;
      case 4: admins.push_back(s); break;
      case 5: crls.push_back(s); break;
      case 7: ous.push_back(s); break;
      case 8: crypto.push_back(s); break;
      default: node.push_back(s); break;
    }
    return true;
  }
};

template <class V>
bool decode_all(const std::vector<Span> &occ, V &v) {
  for (const Span &s : occ)
    if (!pbw::decode(s.p, s.n, v)) return false;
  return true;
}

using Dig = std::array<uint8_t, 32>;

Dig sha(const std::vector<uint8_t> &v) {
  Dig d;
  fgvsha::sha256(v.data(), v.size(), d.data());
  return d;
}

enum : int { R_CLIENT = 2, R_PEER = 3, R_ADMIN = 1, R_ORDERER = 4 };

// a CA of the MSP (root or intermediate), parsed and sanitized at model build
struct CA {
  fgvx::Cert c;
  std::vector<uint8_t> raw2;  // sanitized certificate
  bool root = false;
  uint32_t slot = 0;          // its P-256 key in the key table (pinned)
  std::vector<int> chain;     // itself, its parent, ..., a root (setup's validation chain)
  bool internal = false;      // the parent of an intermediate (certificationTreeInternalNodesMap)
  Dig chain_id{};             // SHA-256 over the sanitized certificates of `chain`
};
constexpr size_t kMaxChain = 8;

// x509 isValid for a CA with `below` intermediates under it + CheckSignatureFrom's rules
// (oracle/msp.py MSP._parent_ok)
bool parent_ok(const fgvx::Cert &p, int64_t now, size_t below) {
  if ((p.version == 3 && !p.bc_valid) || (p.bc_valid && !p.is_ca)) return false;
  if (p.key_usage && !(p.key_usage & (1u << 5))) return false;
  if (!(p.not_before <= now && now <= p.not_after)) return false;
  if (p.bc_valid && p.path_len >= 0 && (int64_t)below > p.path_len) return false;  // TooManyIntermediates
  return true;
}

// child's CA signature as a verify job of the parent's key (false: not a strict DER signature
// with 0 < r, s < n -- the verify fails); Go's ecdsa accepts high S: the low-S equivalent
bool ca_job(const fgvx::Cert &child, uint32_t parent_slot, std::vector<uint8_t> &msgs, std::vector<uint64_t> &moff,
            std::vector<uint32_t> &mlen, std::vector<uint8_t> &sigs, std::vector<uint64_t> &soff,
            std::vector<uint32_t> &slen, std::vector<uint32_t> &slots) {
  uint8_t r[32], s[32];
  if (!fgvx::strict_sig(child.sig(), child.sig_len, r, s) || fgvx::is_zero(r) || fgvx::is_zero(s) || !fgvx::lt_n(r) ||
      !fgvx::lt_n(s))
    return false;
  fgvx::to_low_s(s);
  const std::vector<uint8_t> low = fgvx::der_sig(r, s);
  moff.push_back(msgs.size());
  msgs.insert(msgs.end(), child.tbs(), child.tbs() + child.tbs_len);
  mlen.push_back((uint32_t)child.tbs_len);
  soff.push_back(sigs.size());
  sigs.insert(sigs.end(), low.begin(), low.end());
  slen.push_back((uint32_t)low.size());
  slots.push_back(parent_slot);
  return true;
}
struct RoleOU {
  bool present = false;
  std::string name;
  bool has_cert = false;
  Dig cert{};
};

}  // namespace

struct MspModel {
  bool unsup = false;
  bool sha3 = false;
  std::vector<CA> cas;  // roots first, then intermediates
  std::map<std::string, std::vector<Dig>> ou_ids;
  bool node_ous = false;
  RoleOU role_ou[5];
  std::vector<std::vector<uint8_t>> admins;  // sanitized admin certificates
  std::vector<fgvx::Crl> crls;               // the MSP's revocation lists
  std::vector<std::vector<uint8_t>> crl_ok;  // [crl][ca]: the CA signed the CRL (its SKI = the AKI)

  // the CA whose subject is x's issuer: index, -1 none, -2 several (x509 could build several
  // chains: outside the model)
  int unique_parent(const fgvx::Cert &x, int self) const {
    int found = -1;
    for (size_t j = 0; j < cas.size(); j++)
      if ((int)j != self && x.same_issuer_as_subject_of(cas[j].c)) {
        if (found >= 0) return -2;
        found = (int)j;
      }
    return found;
  }

  // oracle/msp.py MSP.__init__; c->mu held (registers the CA keys, verifies the CA chains on the
  // GPU; c NULL: the sanitizer probe -- no key registration, signatures taken as verified)
  void build(fgv_ctx *c, const std::string &conf) {
    VMspCfg fc;
    if (!pbw::decode(reinterpret_cast<const uint8_t *>(conf.data()), conf.size(), fc)) return fail();
    // setupCRLs (mspimplsetup.go:215-245): a CRL x509.ParseCRL rejects fails the setup; shapes
    // outside oracle/crl.py's model leave the MSP to the reference
    for (const Span &x : fc.crls) {
      fgvx::Crl crl;
      if (fgvx::parse_crl(x.p, x.n, crl) != fgvx::X_OK) return fail();
      crls.push_back(std::move(crl));
    }
    VCryptoCfg cc;
    if (!decode_all(fc.crypto, cc)) return fail();
    if (!cc.idhash.eq("SHA256", 6) && cc.idhash.n) return fail();
    sha3 = cc.fam.eq("SHA3", 4);
    if (fc.roots.empty()) return fail();
    std::vector<uint8_t> keys;
    for (int pass = 0; pass < 2; pass++)
      for (const Span &pem : pass == 0 ? fc.roots : fc.inters) {
        std::vector<uint8_t> der;
        CA a;
        a.root = pass == 0;
        if (fgvx::pem_decode(pem.p, pem.n, der) != fgvx::X_OK) return fail();
        if (fgvx::parse_certificate(std::move(der), a.c) != fgvx::X_OK || a.c.key != fgvx::XK_P256) return fail();
        if (!a.c.is_ca || !a.c.has_ski) return fail();  // finalizeSetupCAs: the MSP would not set up
        if (fgvx::sanitized_raw(a.c, a.raw2) != fgvx::X_OK) return fail();
        keys.insert(keys.end(), a.c.pub, a.c.pub + 64);
        cas.push_back(std::move(a));
      }
    std::vector<uint32_t> slots(cas.size());
    if (c && fgv_keys_register_locked(c, keys.data(), cas.size(), slots.data()) != FGV_OK) return fail();
    for (size_t i = 0; i < cas.size(); i++) cas[i].slot = c ? slots[i] : 0;
    // the validation chains: a root verifies itself; an intermediate walks to a root, checked at
    // its own NotBefore + 1 s; every (child, parent) signature is verified in one GPU pass
    std::vector<uint8_t> msgs, sigs;
    std::vector<uint64_t> moff, soff;
    std::vector<uint32_t> mlen, slen, jslots;
    std::set<std::pair<int, int>> linked;
    auto link = [&](int child, int parent) -> bool {
      if (!linked.insert({child, parent}).second) return true;
      return ca_job(cas[child].c, cas[parent].slot, msgs, moff, mlen, sigs, soff, slen, jslots);
    };
    for (size_t i = 0; i < cas.size(); i++) {
      CA &a = cas[i];
      a.chain.assign(1, (int)i);
      if (a.root) {
        if (!a.c.same_issuer_as_subject_of(a.c) || !link((int)i, (int)i)) return fail();
        continue;
      }
      const int64_t now = a.c.not_before + 1;
      int cur = (int)i;
      while (!cas[cur].root) {
        if (a.chain.size() > kMaxChain) return fail();
        const int p = unique_parent(cas[cur].c, cur);
        if (p < 0 || std::find(a.chain.begin(), a.chain.end(), p) != a.chain.end()) return fail();
        if (!parent_ok(cas[p].c, now, a.chain.size() - 1) || !link(cur, p)) return fail();
        a.chain.push_back(p);
        cur = p;
      }
    }
    if (c && !moff.empty()) {
      std::vector<uint8_t> st(moff.size(), 1);
      if (fgv_verify_msgs_slots_locked(c, msgs.data(), msgs.size(), moff.data(), mlen.data(), sigs.data(), sigs.size(),
                                       soff.data(), slen.data(), jslots.data(), moff.size(), st.data()) != FGV_OK)
        return fail();
      for (uint8_t v : st)
        if (v != 0) return fail();
    }
    // CheckCRLSignature of every CRL by each CA whose SubjectKeyIdentifier is the CRL's
    // AuthorityKeyIdentifier (validateCertAgainstChain consults only those): ECDSA over SHA-256 of
    // the TBSCertList with the re-marshalled (r, s), high S accepted -- one GPU pass
    crl_ok.assign(crls.size(), std::vector<uint8_t>(cas.size(), 0));
    {
      std::vector<uint8_t> cm, cs;
      std::vector<uint64_t> cmo, cso;
      std::vector<uint32_t> cml, csl, csl_slots;
      std::vector<std::pair<size_t, size_t>> who;
      for (size_t i = 0; i < crls.size(); i++)
        for (size_t j = 0; j < cas.size(); j++) {
          const fgvx::Cert &ca = cas[j].c;
          const fgvx::Crl &x = crls[i];
          if (!ca.has_ski || ca.ski_len != x.aki.size() ||
              !std::equal(x.aki.begin(), x.aki.end(), ca.der.begin() + ca.ski_off) || !x.rs_ok)
            continue;
          uint8_t s2[32];
          memcpy(s2, x.s, 32);
          fgvx::to_low_s(s2);
          const std::vector<uint8_t> low = fgvx::der_sig(x.r, s2);
          cmo.push_back(cm.size());
          cm.insert(cm.end(), x.der.begin() + x.tbs_off, x.der.begin() + x.tbs_off + x.tbs_len);
          cml.push_back((uint32_t)x.tbs_len);
          cso.push_back(cs.size());
          cs.insert(cs.end(), low.begin(), low.end());
          csl.push_back((uint32_t)low.size());
          csl_slots.push_back(cas[j].slot);
          who.push_back({i, j});
        }
      std::vector<uint8_t> cst(who.size(), 0);  // (c NULL, the sanitizer probe: taken as verified)
      if (c && !who.empty() &&
          fgv_verify_msgs_slots_locked(c, cm.data(), cm.size(), cmo.data(), cml.data(), cs.data(), cs.size(), cso.data(),
                                       csl.data(), csl_slots.data(), who.size(), cst.data()) != FGV_OK)
        return fail();
      for (size_t q = 0; q < who.size(); q++) crl_ok[who[q].first][who[q].second] = cst[q] == 0;
    }
    // finalizeSetupCAs -> validateCAIdentity: a revoked intermediate CA fails the setup
    for (size_t i = 0; i < cas.size(); i++)
      if (!cas[i].root && revoked(cas[i].c, cas[i].chain[1])) return fail();
    for (CA &a : cas) {
      if (!a.root)
        for (size_t k = 1; k < a.chain.size(); k++) cas[a.chain[k]].internal = true;
      std::vector<uint8_t> cat;
      for (int k : a.chain) cat.insert(cat.end(), cas[k].raw2.begin(), cas[k].raw2.end());
      a.chain_id = sha(cat);
    }
    // certifier of an OU: the chain of the CA whose certificate it is (getCertifiersIdentifier)
    auto certifier = [&](const Span &pem, Dig &out) -> bool {
      std::vector<uint8_t> der;
      if (fgvx::pem_decode(pem.p, pem.n, der) != fgvx::X_OK) return false;
      for (const CA &a : cas)
        if (der == a.c.der) {
          if (!a.root && a.internal) return false;  // getValidationChain(cert, true): parent position 0
          out = a.chain_id;
          return true;
        }
      return false;
    };
    for (const Span &o : fc.ous) {
      VOUIdent id;
      Dig d;
      if (!pbw::decode(o.p, o.n, id) || id.cert.nil() || !certifier(id.cert, d)) return fail();
      ou_ids[id.ou.str()].push_back(d);
    }
    VNodeOUs n;
    if (!decode_all(fc.node, n)) return fail();
    node_ous = n.enable;
    static const int field_role[6] = {0, 0, R_CLIENT, R_PEER, R_ADMIN, R_ORDERER};
    for (int f = 2; f <= 5 && node_ous; f++) {
      if (n.role[f].empty()) continue;
      VOUIdent id;
      if (!decode_all(n.role[f], id)) return fail();
      RoleOU &ro = role_ou[field_role[f]];
      ro.present = true;
      ro.name = id.ou.str();
      if (!id.cert.nil()) {
        if (!certifier(id.cert, ro.cert)) return fail();
        ro.has_cert = true;
      }
    }
    std::vector<fgvx::Cert> acs;
    for (const Span &pem : fc.admins) {
      std::vector<uint8_t> der, raw2;
      fgvx::Cert ac;
      if (fgvx::pem_decode(pem.p, pem.n, der) != fgvx::X_OK) return fail();
      if (fgvx::parse_certificate(std::move(der), ac) != fgvx::X_OK) return fail();
      if (fgvx::sanitized_raw(ac, raw2) != fgvx::X_OK) return fail();
      admins.push_back(std::move(raw2));
      acs.push_back(std::move(ac));
    }
    // postSetupV142 (mspimplsetup.go:684-702; without NodeOUs postSetupV1, :612-624): every admin
    // must Validate -- chain, CRLs, OU identifiers -- or, with NodeOUs, carry the client or the
    // admin OU (hasOURole over GetOrganizationalUnits, empty without a certification chain).
    // Else the MSP does not set up (oracle/msp.py MSP.__init__): outside the model.
    if (!acs.empty()) {
      std::vector<uint8_t> am, as;
      std::vector<uint64_t> amo, aso;
      std::vector<uint32_t> aml, asl, aslots;
      std::vector<int> p1(acs.size());
      for (size_t k = 0; k < acs.size(); k++) {
        const fgvx::Cert &x = acs[k];
        const int64_t now = x.not_before + 1;  // (getUniqueValidationChain, as for any identity)
        if (x.is_ca || x.unhandled_critical || !(x.not_before <= now && now <= x.not_after)) return fail();
        p1[k] = unique_parent(x, -1);
        if (p1[k] < 0) return fail();
        const std::vector<int> &up = cas[p1[k]].chain;
        for (size_t q = 0; q < up.size(); q++)
          if (!parent_ok(cas[up[q]].c, now, q)) return fail();
        if (!ca_job(x, cas[p1[k]].slot, am, amo, aml, as, aso, asl, aslots)) return fail();
      }
      if (c) {  // (c NULL, the sanitizer probe: taken as verified)
        std::vector<uint8_t> st(amo.size(), 1);
        if (fgv_verify_msgs_slots_locked(c, am.data(), am.size(), amo.data(), aml.data(), as.data(), as.size(),
                                         aso.data(), asl.data(), aslots.data(), amo.size(), st.data()) != FGV_OK)
          return fail();
        for (uint8_t v : st)
          if (v != 0) return fail();
      }
      for (size_t k = 0; k < acs.size(); k++) {
        const fgvx::Cert &x = acs[k];
        if (node_ous) {
          if (!has(R_CLIENT, x) && !has(R_ADMIN, x)) return fail();
          continue;
        }
        const CA &issuer = cas[p1[k]];
        if (issuer.internal || !issuer.c.has_ski || revoked(x, p1[k])) return fail();
        if (!ou_ids.empty()) {
          bool any = false;
          for (const std::string &o : x.ous) {
            auto it = ou_ids.find(o);
            if (it != ou_ids.end() && std::find(it->second.begin(), it->second.end(), issuer.chain_id) != it->second.end())
              any = true;
          }
          if (!any) return fail();
        }
      }
    }
  }
  void fail() { unsup = true; }
  // validateCertAgainstChain's CRL loop (mspimplvalidate.go:94-140): c's serial revoked by a CRL
  // that its issuing CA (cas[issuer]) signed
  bool revoked(const fgvx::Cert &c, int issuer) const {
    for (size_t i = 0; i < crls.size(); i++)
      if (crl_ok[i][issuer] && crls[i].revokes(c)) return true;
    return false;
  }
  bool has(int role, const fgvx::Cert &c) const {
    const RoleOU &ro = role_ou[role];
    return ro.present && std::find(c.ous.begin(), c.ous.end(), ro.name) != c.ous.end();
  }
};

struct fgv_msp_cache {
  struct Entry {
    std::string conf;
    std::unique_ptr<MspModel> m;
  };
  std::map<std::string, Entry> by_name;
  bool auto_resolve = true;
};

void fgv_msp_cache_free(fgv_ctx *c) {
  delete c->msp;
  c->msp = nullptr;
}

namespace {

const MspModel *model_of(fgv_ctx *c, const Channel &ch, const std::string &mspid) {
  auto it = ch.config.msp_conf.find(mspid);
  if (!ch.config.present || it == ch.config.msp_conf.end()) return nullptr;
  if (!c->msp) c->msp = new fgv_msp_cache();
  fgv_msp_cache::Entry &e = c->msp->by_name[mspid];
  if (!e.m || e.conf != it->second) {
    e.conf = it->second;
    e.m.reset(new MspModel());
    e.m->build(c, e.conf);
  }
  return e.m.get();
}

struct Pending {
  size_t i;                 // input index
  const MspModel *m;
  fgvx::Cert c;
  int p1 = -1;  // the issuing CA (cas index)
  std::vector<uint8_t> ser;
};

}  // namespace

// c->mu held.  status[i]: FGV_RESOLVE_*.  *registered: identities added to the registry.
int fgv_msp_resolve_locked(fgv_ctx *c, size_t n, const uint8_t *const *ser, const size_t *lens, int *status,
                           size_t *registered) {
  if (registered) *registered = 0;
  if (n == 0) return FGV_OK;
  Channel &ch = fgv_block_channel(c->blk);
  if (ch.dirty) ch.compile();
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  std::vector<Pending> pend;
  std::vector<size_t> undeser;  // DeserializeIdentity fails: registered as undeserializable
  std::unordered_set<std::string> seen;
  for (size_t i = 0; i < n; i++) {
    status[i] = FGV_RESOLVE_KNOWN;
    const Span s{ser[i], (uint32_t)lens[i]};
    if (ch.lookup(s) != -2) continue;  // registered, or not an identity of a channel MSP
    if (!seen.insert(s.str()).second) {  // (a repeat within the call: resolved with the first)
      status[i] = FGV_RESOLVE_REPEAT;
      continue;
    }
    fgvb::VSerializedIdentity sid;
    pbw::decode(s.p, s.n, sid);
    const MspModel *m = model_of(c, ch, sid.mspid.str());
    if (!m || m->unsup) {
      status[i] = FGV_RESOLVE_UNSUPPORTED;
      continue;
    }
    Pending p;
    p.i = i;
    p.m = m;
    p.ser.assign(s.p, s.p + s.n);
    std::vector<uint8_t> der;
    int rc = fgvx::pem_decode(sid.id_bytes.p, sid.id_bytes.n, der);
    if (rc == fgvx::X_OK) rc = fgvx::parse_certificate(std::move(der), p.c);
    if (rc == fgvx::X_UNSUP) {
      status[i] = FGV_RESOLVE_UNSUPPORTED;
      continue;
    }
    if (rc != fgvx::X_OK || p.c.key == fgvx::XK_UNDESERIALIZABLE) {
      undeser.push_back(i);
      continue;
    }
    // getUniqueValidationChain (oracle/msp.py MSP._chain)
    if (p.c.is_ca) {
      status[i] = FGV_RESOLVE_UNSUPPORTED;
      continue;
    }
    const int64_t now = p.c.not_before + 1;
    if (p.c.unhandled_critical || !(p.c.not_before <= now && now <= p.c.not_after)) {
      undeser.push_back(i);
      continue;
    }
    p.p1 = m->unique_parent(p.c, -1);
    if (p.p1 == -2) {
      status[i] = FGV_RESOLVE_UNSUPPORTED;
      continue;
    }
    // the chain above the leaf is the issuer's setup chain (unique parents); each CA on it is
    // checked at this leaf's time and depth (CheckSignatureFrom's rules, validity, MaxPathLen)
    bool ok = p.p1 >= 0;
    if (ok) {
      const std::vector<int> &up = m->cas[p.p1].chain;
      for (size_t k = 0; k < up.size() && ok; k++) ok = parent_ok(m->cas[up[k]].c, now, k);
    }
    if (!ok) {
      undeser.push_back(i);
      continue;
    }
    pend.push_back(std::move(p));
  }
  // the CA signatures over the TBS certificates, one GPU pass (Go's ecdsa accepts high S: the
  // engine's verifier takes the low-S equivalent)
  std::vector<uint8_t> msgs, sigs, vst(pend.size(), 1);
  std::vector<uint64_t> moff, soff;
  std::vector<uint32_t> mlen, slen, slots;
  std::vector<size_t> job(pend.size(), SIZE_MAX);
  for (size_t k = 0; k < pend.size(); k++) {
    const Pending &p = pend[k];
    const size_t j = moff.size();
    if (ca_job(p.c, p.m->cas[p.p1].slot, msgs, moff, mlen, sigs, soff, slen, slots)) job[k] = j;
  }
  std::vector<uint8_t> jst(moff.size(), 1);
  if (!moff.empty()) {
    const int rc = fgv_verify_msgs_slots_locked(c, msgs.data(), msgs.size(), moff.data(), mlen.data(), sigs.data(),
                                                sigs.size(), soff.data(), slen.data(), slots.data(), moff.size(),
                                                jst.data());
    if (rc) return rc;
  }
  // register: verified identities with their Validate / role results, the rest undeserializable
  std::vector<uint8_t> keys;
  struct Reg {
    size_t i;
    fgv_identity_info info;
    const std::vector<std::string> *ous;  // GetOrganizationalUnits: the subject OUs ...
    Dig certifier;                        // ... each with the chain above the identity
  };
  std::vector<Reg> regs;
  for (size_t k = 0; k < pend.size(); k++) {
    const Pending &p = pend[k];
    if (job[k] == SIZE_MAX || jst[job[k]] != 0) {
      undeser.push_back(p.i);
      continue;
    }
    std::vector<uint8_t> raw2;
    if (fgvx::sanitized_raw(p.c, raw2) != fgvx::X_OK) {
      status[p.i] = FGV_RESOLVE_UNSUPPORTED;
      continue;
    }
    const MspModel &m = *p.m;
    Reg g{p.i, fgv_identity_info{}, &p.c.ous, p.m->cas[p.p1].chain_id};
    const Dig dg = sha(raw2);
    memcpy(g.info.id_digest, dg.data(), 32);
    // Validate: the issuer must be a leaf of the certification tree (its SKI exists: setup),
    // then the OUs (validateIdentityOUsV142) with the chain above the identity as certifier
    const CA &issuer = m.cas[p.p1];
    bool valid = !issuer.internal && issuer.c.has_ski;
    if (valid && !m.crls.empty() && m.revoked(p.c, p.p1)) valid = false;  // revoked (CRLs)
    const Dig &cid = issuer.chain_id;
    if (valid && !m.ou_ids.empty()) {
      bool any = false;
      for (const std::string &o : p.c.ous) {
        auto it = m.ou_ids.find(o);
        if (it != m.ou_ids.end() && std::find(it->second.begin(), it->second.end(), cid) != it->second.end()) any = true;
      }
      valid = any;
    }
    if (valid && m.node_ous) {
      int cnt = 0;
      static const int order[4] = {R_CLIENT, R_PEER, R_ADMIN, R_ORDERER};  // (a later role's identical OU wins)
      for (const std::string &o : p.c.ous) {
        const RoleOU *hit = nullptr;
        for (int r : order)
          if (m.role_ou[r].present && m.role_ou[r].name == o) hit = &m.role_ou[r];
        if (!hit) continue;
        if (hit->has_cert && hit->cert != cid) {
          valid = false;
          break;
        }
        if (++cnt > 1) break;
      }
      if (cnt != 1) valid = false;
    }
    uint32_t roles = valid ? 1u : 0u;
    const bool admin_listed = std::find(m.admins.begin(), m.admins.end(), raw2) != m.admins.end();
    if (admin_listed || (valid && m.node_ous && m.has(R_ADMIN, p.c))) roles |= 1u << R_ADMIN;
    for (int r : {R_CLIENT, R_PEER, R_ORDERER})
      if (valid && m.node_ous && m.has(r, p.c)) roles |= 1u << r;
    g.info.valid = valid;
    g.info.roles = roles;
    g.info.hash_family = m.sha3 ? FGV_HASH_SHA3 : FGV_HASH_SHA2;
    g.info.key_type = p.c.key == fgvx::XK_P256 ? FGV_KEY_P256 : p.c.key == fgvx::XK_P384 ? FGV_KEY_P384 : FGV_KEY_OTHER;
    if (g.info.key_type == FGV_KEY_P256) memcpy(g.info.pubkey, p.c.pub, 64);
    if (g.info.key_type == FGV_KEY_P384) memcpy(g.info.pubkey_p384, p.c.pub384, 96);  // (round 6)
    regs.push_back(g);
  }
  // every new P-256 key in one registration: comb tables for the roles that sign often (peers,
  // orderers, admins), the variable-base kernels for the others until they are promoted by use
  std::vector<uint8_t> want;
  for (const Reg &g : regs)
    if (g.info.key_type == FGV_KEY_P256) {
      keys.insert(keys.end(), g.info.pubkey, g.info.pubkey + 64);
      want.push_back(fgv_roles_want_comb(g.info.roles) ? 1 : 0);
    }
  std::vector<uint32_t> kslots(keys.size() / 64);
  if (!kslots.empty()) {
    const int rc = fgv_keys_register_locked(c, keys.data(), kslots.size(), kslots.data(), want.data());
    if (rc) return rc;
  }
  size_t kq = 0, nreg = 0;
  for (const Reg &g : regs) {
    int32_t slot = g.info.key_type == FGV_KEY_P256 ? (int32_t)kslots[kq++] : -1;
    if (g.info.key_type == FGV_KEY_P384) {  // a P-384 leaf: its comb in the P-384 key table (p384.hip)
      uint32_t k;
      const int rc = fgv_p384_key_locked(c, g.info.pubkey_p384, &k);
      if (rc) return rc;
      slot = (int32_t)(KEY_P384_FLAG | k);
    }
    if (fgv_block_add_identity(c->blk, ser[g.i], lens[g.i], slot, &g.info) == FGV_OK) {
      nreg++;
      std::vector<const char *> op;
      std::vector<size_t> ol, cl;
      std::vector<const uint8_t *> cp;
      for (const std::string &o : *g.ous) {
        op.push_back(o.data());
        ol.push_back(o.size());
        cp.push_back(g.certifier.data());
        cl.push_back(g.certifier.size());
      }
      fgv_block_identity_ous(c->blk, ser[g.i], lens[g.i], op.size(), op.data(), ol.data(), cp.data(), cl.data());
    }
    status[g.i] = FGV_RESOLVE_OK;
  }
  for (size_t i : undeser) {
    fgv_identity_info info{};
    info.key_type = FGV_KEY_UNDESERIALIZABLE;
    info.roles = 0;
    if (fgv_block_add_identity(c->blk, ser[i], lens[i], -1, &info) == FGV_OK) nreg++;
    status[i] = FGV_RESOLVE_FAILED;
  }
  if (registered) *registered = nreg;
  return FGV_OK;
}

// the misses a batch of blocks names (fgv_block_misses), resolved; c->mu held
int fgv_msp_resolve_blocks_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                  size_t *registered) {
  if (registered) *registered = 0;
  std::vector<std::string> miss;
  fgv_block_misses(c->blk, nblocks, blocks, lens, miss);
  if (miss.empty()) return FGV_OK;
  std::vector<const uint8_t *> p(miss.size());
  std::vector<size_t> l(miss.size());
  for (size_t i = 0; i < miss.size(); i++) {
    p[i] = reinterpret_cast<const uint8_t *>(miss[i].data());
    l[i] = miss[i].size();
  }
  std::vector<int> st(miss.size());
  return fgv_msp_resolve_locked(c, miss.size(), p.data(), l.data(), st.data(), registered);
}

bool fgv_msp_auto(fgv_ctx *c) { return !c->msp || c->msp->auto_resolve; }

extern "C" {

int fgv_msp_resolve(fgv_ctx *c, size_t n, const uint8_t *const *serialized, const size_t *lens, int *status) {
  if (!c || (n && (!serialized || !lens || !status))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_msp_resolve_locked(c, n, serialized, lens, status, nullptr);
}

int fgv_msp_resolve_blocks(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                           size_t *registered) {
  if (!c || (nblocks && (!blocks || !lens))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_msp_resolve_blocks_locked(c, nblocks, blocks, lens, registered);
}

int fgv_set_auto_resolve(fgv_ctx *c, int on) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->msp) c->msp = new fgv_msp_cache();
  c->msp->auto_resolve = on != 0;
  return FGV_OK;
}

int fgv_msp_identity(fgv_ctx *c, const uint8_t *serialized, size_t len, fgv_identity_info *out) {
  if (!c || !serialized || !out) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  Channel &ch = fgv_block_channel(c->blk);
  if (ch.dirty) ch.compile();
  fgvb::VSerializedIdentity sid;
  if (!pbw::decode(serialized, len, sid)) return FGV_ESTATE;
  uint64_t h = fgvb::hash_bytes(sid.mspid.p, sid.mspid.n);
  h = fgvb::hash_bytes(sid.id_bytes.p, sid.id_bytes.n, h ^ 0xA5);
  auto range = ch.ident_index.equal_range(h);
  for (auto it = range.first; it != range.second; ++it) {
    const Ident &I = ch.idents[it->second];
    if (!sid.mspid.eq(I.mspid.data(), I.mspid.size()) || !sid.id_bytes.eq(I.id_bytes.data(), I.id_bytes.size()))
      continue;
    *out = fgv_identity_info{};
    out->key_type = I.kind;
    out->hash_family = I.hash3 ? FGV_HASH_SHA3 : FGV_HASH_SHA2;
    out->valid = I.valid;
    out->roles = I.roles_known ? I.roles : FGV_ROLES_UNKNOWN;
    memcpy(out->pubkey, I.pub, 64);
    memcpy(out->pubkey_p384, I.pub384, 96);
    memcpy(out->id_digest, I.digest, 32);
    return FGV_OK;
  }
  return FGV_ESTATE;
}

}  // extern "C"

// Sanitizer probe (tools/sanitize/harness.cpp): FabricMSPConfig bytes through the MSP model's
// parse (visitors, root / admin / OU certificates) without the key registration; 1 = modelled
uint64_t fgv_msp_config_probe(const uint8_t *conf, size_t n) {
  MspModel m;
  m.build(nullptr, std::string(reinterpret_cast<const char *>(conf), n));
  return m.unsup ? 0 : 1 + m.cas.size() * 16 + m.admins.size() * 256;
}
