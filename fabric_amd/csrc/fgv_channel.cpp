// fgv_channel.cpp -- compiling the channel model (fgv_channel.h): channel configuration walk,
// signature-policy compilation (cauthdsl.compile shape), ImplicitMeta thresholds, chaincode and
// collection endorsement policies.  Host code, run when the model changes.
#include "fgv_channel.h"

#include <algorithm>

namespace fgvb {

// ------------------------------------------------------------------ signature policies
namespace {

struct VNOutOf {
  int32_t n = 0;
  std::vector<Span> rules;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { n = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { rules.push_back(s); return true; }
};
struct VSigPolicyRaw {  // SignaturePolicy oneof {signed_by = 1, n_out_of = 2}: the last member wins
  int which = 0;
  int32_t signed_by = 0;
  std::vector<Span> noutof;  // merged occurrences
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { which = 1; signed_by = pbw::as_int32(v); noutof.clear(); }
  bool on_len(uint32_t, Span s) {
    if (which != 2) noutof.clear();
    which = 2;
    noutof.push_back(s);
    return true;
  }
};
struct VSPE {  // SignaturePolicyEnvelope {version 1, rule 2, identities 3}
  int32_t version = 0;
  bool has_rule = false;
  std::vector<Span> rule;
  std::vector<Span> identities;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_MSG : f == 3 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { version = pbw::as_int32(v); }
  bool on_len(uint32_t f, Span s) {
    if (f == 2) { has_rule = true; rule.push_back(s); }
    else identities.push_back(s);
    return true;
  }
};
struct VAppPolicy {  // ApplicationPolicy oneof {signature_policy 1, channel_config_policy_reference 2}
  int which = 0;
  std::vector<Span> spe;
  Span ref;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_MSG : f == 2 ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    if (f == 1) {
      if (which != 1) spe.clear();
      which = 1;
      spe.push_back(s);
    } else {
      which = 2;
      spe.clear();
      ref = s;
    }
    return true;
  }
};

bool decode_sigpolicy(const std::vector<Span> &occ, VSigPolicyRaw &out) {
  for (const Span &s : occ)
    if (!pbw::decode(s.p, s.n, out)) return false;
  return true;
}

// cauthdsl.compile shape; node index, or -1 on a compile error
int build_node(Policy &P, const std::vector<Span> &occ, bool &wire_ok, int depth) {
  if (depth > 1000) { wire_ok = false; return -1; }
  VSigPolicyRaw raw;
  if (!decode_sigpolicy(occ, raw)) { wire_ok = false; return -1; }
  PNode node;
  if (raw.which == 1) {
    node.type = 2;
    if (raw.signed_by < 0 || raw.signed_by >= (int32_t)P.prin_off.size()) return -1;
    node.principal = raw.signed_by;
  } else if (raw.which == 2) {
    node.type = 1;
    VNOutOf no;
    for (const Span &s : raw.noutof)
      if (!pbw::decode(s.p, s.n, no)) { wire_ok = false; return -1; }
    node.n = no.n;
    std::vector<int> kids;  // sub-rules decode eagerly (proto.Unmarshal) before compile errors
    bool compile_fail = false;
    for (const Span &r : no.rules) {
      std::vector<Span> one{r};
      int k = build_node(P, one, wire_ok, depth + 1);
      if (!wire_ok) return -1;
      if (k < 0) compile_fail = true;
      kids.push_back(k);
    }
    if (compile_fail) return -1;
    node.kids = kids;
  } else {
    return -1;  // "Unknown type" (a nil rule is the caller's "Empty policy element")
  }
  P.nodes.push_back(node);
  return (int)P.nodes.size() - 1;
}

struct VOrgUnit {  // OrganizationUnit {msp_identifier 1, organizational_unit_identifier 2, certifiers_identifier 3}
  Span mspid, ou, certifier;
  pbw::Kind kind(uint32_t f) { return f <= 2 && f ? pbw::K_STRING : f == 3 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    (f == 1 ? mspid : f == 2 ? ou : certifier) = s;
    return true;
  }
};
struct VAnonymity {  // MSPIdentityAnonymity {anonymity_type 1}
  int32_t type = 0;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { type = pbw::as_int32(v); }
  bool on_len(uint32_t, Span) { return true; }
};
struct VCombined {  // CombinedPrincipal {principals 1 (repeated MSPPrincipal)}: decoded eagerly
  std::vector<VPrincipal> prs;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    VPrincipal p;
    if (!pbw::decode(s.p, s.n, p)) return false;
    prs.push_back(p);
    return true;
  }
};

// collectPrincipals (msp/mspimpl.go:440-471) + each leaf's compiled check; a COMBINED that does
// not decode or holds no principal is an error for every identity (a NEVER leaf: the AND of the
// leaves fails).  false: nesting beyond the engine's bound (outside the model).
bool compile_principal(Channel &ch, int32_t cls, const Span &body, std::vector<Prin> &out, bool &needs_roles,
                       int depth) {
  Prin p;
  if (cls == 4) {  // COMBINED (MSP >= v1.1)
    if (depth > 16) return false;
    VCombined cp;
    if (!pbw::decode(body.p, body.n, cp) || cp.prs.empty()) {
      out.push_back(p);
      return true;
    }
    for (const VPrincipal &q : cp.prs)
      if (!compile_principal(ch, q.cls, q.principal, out, needs_roles, depth + 1)) return false;
    return true;
  }
  if (cls == 0) {  // ROLE
    VMSPRole role;
    if (pbw::decode(body.p, body.n, role) && role.role >= 0 && role.role <= 4) {  // ("invalid MSP role type")
      p.kind = PR_ROLE;
      p.msp = ch.intern(role.mspid.str());
      p.role = role.role;
      needs_roles |= role.role != 0;
    }
  } else if (cls == 1) {  // ORGANIZATION_UNIT
    VOrgUnit ou;
    if (pbw::decode(body.p, body.n, ou)) {
      p.kind = PR_OU;
      p.msp = ch.intern(ou.mspid.str());
      p.ou = ch.ou_intern(std::string_view(reinterpret_cast<const char *>(ou.certifier.p), ou.certifier.n),
                          std::string_view(reinterpret_cast<const char *>(ou.ou.p), ou.ou.n));
    }
  } else if (cls == 2) {  // IDENTITY: the identity's MSP deserializes the principal
    const int j = ch.lookup(body);
    if (j >= 0) {
      p.kind = PR_IDENTITY;
      p.msp = ch.idents[j].msp;
      p.canon = ch.idents[j].canon;
    } else if (j == -2) {
      p.kind = PR_UNRESOLVED;
      ch.unresolved_principals.push_back(body.str());
    }
  } else if (cls == 3) {  // ANONYMITY: NOMINAL holds for any identity, ANONYMOUS for none
    VAnonymity an;
    if (pbw::decode(body.p, body.n, an) && an.type == 0) p.kind = PR_NOMINAL;
  }
  out.push_back(p);
  return true;
}

}  // namespace

// a SignaturePolicyEnvelope (all occurrences merged) -> Policy; check_version: the channel-config
// provider accepts version 0 only (cauthdsl.NewPolicy), application policies skip the check
static Policy compile_spe(Channel &ch, const std::vector<Span> &occ, bool check_version) {
  Policy P;
  P.kind = PK_SIG;
  VSPE spe;
  for (const Span &s : occ)
    if (!pbw::decode(s.p, s.n, spe)) return P;  // unmarshal error -> evaluation error
  std::vector<VPrincipal> prs(spe.identities.size());
  for (size_t i = 0; i < spe.identities.size(); i++)
    if (!pbw::decode(spe.identities[i].p, spe.identities[i].n, prs[i])) return P;
  bool in_model = true;
  for (const VPrincipal &pr : prs) {
    P.prin_off.push_back((uint32_t)P.prins.size());
    in_model &= compile_principal(ch, pr.cls, pr.principal, P.prins, P.needs_roles, 0);
    P.prin_cnt.push_back((uint32_t)P.prins.size() - P.prin_off.back());
  }
  bool wire_ok = true;
  int root = -1;
  if (spe.has_rule) root = build_node(P, spe.rule, wire_ok, 0);
  if (!wire_ok) {
    Policy bad;
    bad.kind = PK_SIG;
    return bad;
  }
  if (!in_model) { P.kind = PK_UNSUP; return P; }
  if (check_version && spe.version != 0) { P.kind = PK_UNSUP; return P; }
  P.decode_ok = true;
  P.root = root;
  P.compile_ok = root >= 0;
  return P;
}

static int push_policy(Channel &ch, Policy P) {
  ch.policies.push_back(std::move(P));
  return (int)ch.policies.size() - 1;
}

int Channel::compile_app(const std::string &bytes) {
  VAppPolicy ap;
  if (!pbw::decode(reinterpret_cast<const uint8_t *>(bytes.data()), bytes.size(), ap)) return 0;
  if (ap.which == 1) return push_policy(*this, compile_spe(*this, ap.spe, false));
  if (ap.which != 2) return 0;  // unsupported policy type -> evaluation error
  if (!config.present || config.unsupported) {
    Policy u;
    u.kind = PK_UNSUP;
    return push_policy(*this, u);
  }
  std::string ref = ap.ref.str();  // ManagerImpl.GetPolicy on the root "Channel" manager
  if (!ref.empty() && ref[0] == '/') {
    static const std::string root = "/Channel/";
    if (ref.compare(0, root.size(), root) != 0) return 0;
    ref = ref.substr(root.size());
  }
  auto it = chan_idx.find(ref);
  return (ref.empty() || it == chan_idx.end()) ? 0 : it->second;
}

void Channel::compile() {
  unresolved_principals.clear();
  policies.clear();
  policies.push_back(Policy());  // [0]: reject
  chan_idx.clear();
  ccs.clear();
  implicit_ep.clear();
  known_msps.clear();
  for (const Ident &I : idents) known_msps.insert(I.msp);
  for (const std::string &m : declared_msps) known_msps.insert(intern(m));
  if (config.present) {
    for (const auto &kv : config.msps) known_msps.insert(intern(kv.first));
    for (const auto &kv : config.policies) {
      chan_idx[kv.first] = (int)policies.size();
      policies.push_back(Policy());
    }
    for (const auto &kv : config.policies) {
      const RawChanPolicy &rp = kv.second;
      Policy P;
      if (rp.type == 1) {
        std::vector<Span> one{Span{reinterpret_cast<const uint8_t *>(rp.value.data()), (uint32_t)rp.value.size()}};
        P = compile_spe(*this, one, true);
      } else if (rp.type == 3) {  // implicitmeta.go:27-60
        P.kind = PK_IMPLICIT;
        for (const std::string &s : rp.subs) {
          auto it = chan_idx.find(s);
          P.subs.push_back(it == chan_idx.end() ? 0 : it->second);
        }
        const int n = (int)P.subs.size();
        P.threshold = rp.rule == 0 ? 1 : rp.rule == 1 ? n : rp.rule == 2 ? n / 2 + 1 : 0;
        if (n == 0) P.threshold = 0;
      } else {
        P.kind = PK_UNSUP;
      }
      if (config.unsupported) P.kind = PK_UNSUP;
      policies[chan_idx[kv.first]] = std::move(P);
    }
    for (const auto &kv : chan_idx) {  // ImplicitMeta over ImplicitMeta: outside the model
      Policy &P = policies[kv.second];
      if (P.kind != PK_IMPLICIT) continue;
      for (int s : P.subs) {
        if (policies[s].kind == PK_IMPLICIT) P.kind = PK_UNSUP;
        P.needs_roles |= policies[s].needs_roles;
      }
    }
    // implicit org collections (deployedcc_infoprovider.go:270-305): the org's Endorsement
    // policy, else SignedByAnyMember([mspid])
    if (!config.unsupported)
      for (const auto &kv : config.app_orgs) {
        auto it = chan_idx.find("Application/" + kv.second + "/Endorsement");
        if (it != chan_idx.end()) {
          implicit_ep[kv.first] = it->second;
          continue;
        }
        Policy P;
        P.kind = PK_SIG;
        P.decode_ok = P.compile_ok = true;
        Prin pr;
        pr.kind = PR_ROLE;
        pr.msp = intern(kv.first);
        P.prin_off.push_back(0);
        P.prin_cnt.push_back(1);
        P.prins.push_back(pr);
        PNode sb;
        sb.type = 2;
        sb.principal = 0;
        P.nodes.push_back(sb);
        PNode no;
        no.type = 1;
        no.n = 1;
        no.kids.push_back(0);
        P.nodes.push_back(no);
        P.root = 1;
        implicit_ep[kv.first] = push_policy(*this, std::move(P));
      }
  }
  // SHA3 MSPs (from the config) mark their identities
  for (Ident &I : idents) {
    auto it = config.msps.find(I.mspid);
    if (it != config.msps.end() && it->second) I.hash3 = true;
  }
  for (const auto &kv : ccdefs) {
    const CCDef &d = kv.second;
    CCInfo c;
    if (d.plugin.empty() || d.policy.empty()) {
      c.status = 1;  // getCDataForCC: plugin / policy must be set -> INVALID_CHAINCODE
    } else if (d.plugin != "vscc" || (d.flags & FGV_CC_KEY_LEVEL_EP)) {
      c.status = 2;
    } else {
      c.ep = compile_app(d.policy);
      c.colls_known = (d.flags & FGV_CC_COLLECTIONS_KNOWN) != 0;
      for (const auto &cl : d.colls) c.colls[cl.first] = cl.second.empty() ? -1 : compile_app(cl.second);
    }
    c.has_vp = kvmeta_ns.count(kv.first) != 0;
    ccs[kv.first] = std::move(c);
  }
  // key-level validation parameters: toApplicationPolicyTranslator (builtin/v20/
  // validation_logic.go:50-66) wraps the SignaturePolicyEnvelope as an ApplicationPolicy, which
  // the evaluator takes without the version check; an envelope that does not unmarshal fails
  // the translation
  // (identical parameters share one compiled policy: a state typically holds few distinct ones)
  kvmeta_pi.clear();
  std::unordered_map<std::string_view, int> by_bytes;
  for (const auto &kv : kvmeta) {
    auto hit = by_bytes.find(kv.second);
    if (hit != by_bytes.end()) {
      kvmeta_pi[kv.first] = hit->second;
      continue;
    }
    std::vector<Span> one{Span{reinterpret_cast<const uint8_t *>(kv.second.data()), (uint32_t)kv.second.size()}};
    Policy P = compile_spe(*this, one, false);
    const int pi = (P.kind == PK_SIG && !P.decode_ok) ? -3 : push_policy(*this, std::move(P));
    by_bytes.emplace(kv.second, pi);
    kvmeta_pi[kv.first] = pi;
  }
  dirty = false;
}

// ------------------------------------------------------------------ channel configuration
namespace {

struct VMapEntry {  // map<string, Msg> entry {key = 1, value = 2}
  Span key;
  std::vector<Span> value;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_STRING : f == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    if (f == 1) key = s;
    else value.push_back(s);
    return true;
  }
};
struct VConfigGroup {  // {version 1, groups 2, values 3, policies 4, mod_policy 5}
  std::vector<Span> groups, values, policies;
  pbw::Kind kind(uint32_t f) {
    return f == 1 ? pbw::K_VARINT : (f >= 2 && f <= 4) ? pbw::K_REP_MSG : f == 5 ? pbw::K_STRING : pbw::K_NONE;
  }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    if (f == 2) groups.push_back(s);
    else if (f == 3) values.push_back(s);
    else if (f == 4) policies.push_back(s);
    return true;
  }
};
struct VConfigValue {  // {version 1, value 2, mod_policy 3}
  Span value;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_BYTES : f == 3 ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) { if (f == 2) value = s; return true; }
};
struct VConfigPolicy {  // {version 1, policy 2, mod_policy 3}
  std::vector<Span> policy;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_MSG : f == 3 ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) { if (f == 2) policy.push_back(s); return true; }
};
struct VPolicyMsg {  // Policy {type 1, value 2}
  int32_t type = 0;
  Span value;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { type = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { value = s; return true; }
};
struct VImplicitMeta {  // {sub_policy 1, rule 2}
  Span sub;
  int32_t rule = 0;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_STRING : f == 2 ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { rule = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { sub = s; return true; }
};
struct VMSPConfig {  // {type 1, config 2}
  int32_t type = 0;
  Span config;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { type = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { config = s; return true; }
};
struct VFabricMSPConfig {  // {name 1, ..., crypto_config 8, ...}
  Span name;
  std::vector<Span> crypto;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_STRING : f == 8 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) {
    if (f == 1) name = s;
    else crypto.push_back(s);
    return true;
  }
};
struct VCrypto {  // FabricCryptoConfig {signature_hash_family 1, identity_identifier_hash_function 2}
  Span family;
  pbw::Kind kind(uint32_t f) { return (f == 1 || f == 2) ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t f, Span s) { if (f == 1) family = s; return true; }
};
struct VConfig {  // Config {sequence 1, channel_group 2}
  std::vector<Span> group;
  pbw::Kind kind(uint32_t f) { return f == 1 ? pbw::K_VARINT : f == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) { group.push_back(s); return true; }
};

template <class V>
bool decode_all(const std::vector<Span> &occ, V &v) {
  for (const Span &s : occ)
    if (!pbw::decode(s.p, s.n, v)) return false;
  return true;
}

// map entries: the last entry of a key wins (Go map unmarshal)
bool entries(const std::vector<Span> &raw, std::map<std::string, std::vector<Span>> &out) {
  for (const Span &e : raw) {
    VMapEntry me;
    if (!pbw::decode(e.p, e.n, me)) return false;
    out[me.key.str()] = me.value;
  }
  return true;
}

bool walk(const std::vector<Span> &occ, const std::string &path, const std::string &parent, RawConfig &out, int depth) {
  if (depth > 64) return false;
  VConfigGroup g;
  if (!decode_all(occ, g)) return false;
  std::map<std::string, std::vector<Span>> groups, values, pols;
  if (!entries(g.groups, groups) || !entries(g.values, values) || !entries(g.policies, pols)) return false;
  auto mv = values.find("MSP");
  if (mv != values.end()) {
    VConfigValue cv;
    VMSPConfig mc;
    VFabricMSPConfig fc;
    VCrypto cc;
    if (!decode_all(mv->second, cv) || !pbw::decode(cv.value.p, cv.value.n, mc)) return false;
    if (mc.type == 0) {  // X.509 MSP (idemix MSPs hold no X.509 identities: left out)
      if (!pbw::decode(mc.config.p, mc.config.n, fc) || !decode_all(fc.crypto, cc)) return false;
      const std::string name = fc.name.str(), fam = cc.family.str();
      if (fam != "SHA2" && fam != "SHA3") out.unsupported = true;
      out.msps[name] = fam == "SHA3";
      out.msp_conf[name] = mc.config.str();  // (the cache-miss path builds its MSP model from it)
      if (parent == "Application") out.app_orgs[name] = path.substr(path.rfind('/') + 1);
    }
  }
  for (const auto &kv : pols) {
    VConfigPolicy cp;
    VPolicyMsg pm;
    if (!decode_all(kv.second, cp) || !decode_all(cp.policy, pm)) return false;
    RawChanPolicy rp;
    rp.type = pm.type;
    rp.value = pm.value.str();
    if (pm.type == 3) {
      VImplicitMeta im;
      if (!pbw::decode(pm.value.p, pm.value.n, im)) return false;
      rp.rule = im.rule;
      for (const auto &c : groups) rp.subs.push_back((path.empty() ? "" : path + "/") + c.first + "/" + im.sub.str());
    }
    out.policies[(path.empty() ? "" : path + "/") + kv.first] = std::move(rp);
  }
  const std::string me = path.empty() ? std::string() : path.substr(path.rfind('/') + 1);
  for (const auto &kv : groups)
    if (!walk(kv.second, (path.empty() ? "" : path + "/") + kv.first, path.empty() ? std::string("") : me, out, depth + 1))
      return false;
  return true;
}

}  // namespace

bool parse_channel_config(const uint8_t *p, size_t n, RawConfig &out) {
  out = RawConfig();
  VConfig c;
  if (!pbw::decode(p, n, c)) return false;
  if (!walk(c.group, "", "", out, 0)) return false;
  out.present = true;
  return true;
}

}  // namespace fgvb
