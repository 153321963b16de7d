// fgv_channel.h -- the channel model the committer validates against (host side of libfgv.so):
// MSP identities, channel-config policies, chaincode / collection endorsement policies.  It is
// what the reference's validator reads through its channel resources, restated:
//   identities   msp/mspmgrimpl.go:75-100 (DeserializeIdentity), msp/identities.go:170-227
//                (Verify, hash family), msp/mspimpl.go:331-376 + 477-660 (SatisfiesPrincipal by
//                role: the MSP layer's answer per role arrives with the identity)
//   policies     common/cauthdsl/cauthdsl.go:24-92 (signature policies),
//                common/policies/implicitmeta.go:27-104 (ImplicitMeta), policy.go:330-358
//                (GetPolicy path resolution; sub-manager policies folded into the parent map),
//                core/policy/application.go:139-163 (ApplicationPolicy: signature policy or
//                channel config policy reference)
//   chaincodes   plugindispatcher/dispatcher.go:237-275 (ValidationInfo: plugin + policy; an
//                empty one -> INVALID_CHAINCODE), core/chaincode/lifecycle/
//                deployedcc_infoprovider.go:270-382 (collection EPs, implicit org collections)
// The raw inputs are kept; compile() turns them into a flat policy table whenever they change.
#pragma once
#include <stdint.h>

#include <deque>
#include <map>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_visitors.h"

namespace fgvb {

struct Ident {
  std::string mspid, id_bytes;
  int32_t key_slot = -1;        // P-256 key table slot (FGV_KEY_P256 only)
  uint8_t kind = FGV_KEY_OTHER; // FGV_KEY_*
  bool hash3 = false;           // the MSP hashes with SHA3 (identities.go:219-227)
  bool valid = false;           // msp Validate() result
  bool roles_known = false;
  uint32_t roles = 0;           // bit r: satisfies ROLE principal r of its own MSP
  uint32_t canon = 0;           // dedup identity id: Mspid + Id (Id = hex SHA-256(cert))
  int32_t msp = -1;             // interned Mspid
  uint8_t digest[32] = {};      // identity Id (SHA-256 of the certificate)
  uint8_t pub[64] = {};         // P-256 X || Y (FGV_KEY_P256)
  uint8_t pub384[96] = {};      // P-384 X || Y (FGV_KEY_P384; key_slot = KEY_P384_FLAG | its table index)
  // GetOrganizationalUnits (msp/identities.go): (OU identifier, certifiers identifier) pairs,
  // interned by Channel::ou_intern; unknown unless the MSP cache miss or fgv_msp_identity_ous
  // gave them
  bool ous_known = false;
  std::vector<int32_t> ous;
  // Verify outcome class: 0 = verified on the GPU, 1 = always fails (RSA, F5), 2 = outside
  // the engine (P-384, SHA3 MSP)
  int verify_class() const {
    if (kind == FGV_KEY_OTHER) return 1;
    if (kind != FGV_KEY_P256 || hash3 || key_slot < 0) return 2;
    return 0;
  }
  // the same for the committer's creator and endorsement signatures, whose digests follow the
  // identity's hash family (SHA3 MSPs included since round 5: the SHA3-256 digest pass) and whose
  // P-384 keys are verified per item (round 6, p384.hip); the other Verify callers (orderer
  // signatures) keep SHA3 and P-384 identities outside the engine
  int verify_class_tx() const {
    if (kind == FGV_KEY_OTHER) return 1;
    if ((kind != FGV_KEY_P256 && kind != FGV_KEY_P384) || key_slot < 0) return 2;
    return 0;
  }
};

struct PNode {
  int type = 0;  // 1 NOutOf, 2 SignedBy
  int32_t n = 0;
  int principal = -1;  // SignedBy: index of the envelope's principal (Policy::prin_off / prin_cnt)
  std::vector<int> kids;
};
// One leaf principal of an MSPPrincipal after collectPrincipals (msp/mspimpl.go:440-471, a
// COMBINED principal flattened into its leaves, all of which must hold), compiled for MSP v1.4.3
// (satisfiesPrincipalInternalV142 -> V13 -> PreV13, mspimpl.go:477-660).
enum PrinKind : uint8_t {
  PR_ROLE = 0,        // MSPRole: same MSP, MEMBER = Validate, other roles from the identity's role bits
  PR_IDENTITY = 1,    // SerializedIdentity: the same sanitized certificate (Mspid + Id), and Validate
  PR_OU = 2,          // OrganizationUnit: same MSP, Validate, an OU with that identifier and certifier
  PR_NOMINAL = 3,     // MSPIdentityAnonymity NOMINAL: every identity
  PR_NEVER = 4,       // an error for every identity (undecodable, unknown class, ANONYMOUS, ...)
  PR_UNRESOLVED = 5,  // IDENTITY of a channel MSP not yet deserialized: outside the model until resolved
};
struct Prin {
  uint8_t kind = PR_NEVER;
  int32_t msp = -1;    // ROLE / OU: interned MspIdentifier
  int32_t role = 0;    // ROLE
  uint32_t canon = 0;  // IDENTITY
  int32_t ou = -1;     // OU: Channel::ou_intern(certifier, identifier)
};
enum PolKind : uint8_t { PK_REJECT = 0, PK_SIG = 1, PK_IMPLICIT = 2, PK_UNSUP = 3 };
struct Policy {
  uint8_t kind = PK_REJECT;
  bool decode_ok = false, compile_ok = false;  // PK_SIG: rule decoded / compiled
  std::vector<PNode> nodes;
  int root = -1;
  // envelope principal i = the leaves prins[prin_off[i] .. prin_off[i] + prin_cnt[i])
  std::vector<uint32_t> prin_off, prin_cnt;
  std::vector<Prin> prins;
  bool needs_roles = false;             // a ROLE leaf with a role other than MEMBER
  int threshold = 0;                    // PK_IMPLICIT
  std::vector<int> subs;                // PK_IMPLICIT: policy indices (0 = reject)
};

// channel configuration, parsed once per fgv_channel_config call
struct RawChanPolicy {
  int32_t type = 0;            // common.Policy.type: 1 SIGNATURE, 3 IMPLICIT_META
  std::string value;
  int32_t rule = 0;            // IMPLICIT_META
  std::vector<std::string> subs;  // IMPLICIT_META: child-group sub-policy paths
};
struct RawConfig {
  bool present = false;
  bool unsupported = false;                       // e.g. an MSP with an unknown hash family
  std::map<std::string, RawChanPolicy> policies;  // "Application/org1/Endorsement" (relative to /Channel)
  std::map<std::string, bool> msps;               // MSP name -> SHA3
  std::map<std::string, std::string> msp_conf;    // MSP name -> FabricMSPConfig bytes (fgv_msp.cpp)
  std::map<std::string, std::string> app_orgs;    // mspid -> application org group name
};
bool parse_channel_config(const uint8_t *p, size_t n, RawConfig &out);

struct CCDef {  // lifecycle ValidationInfo + collection configs of one namespace
  std::string plugin, policy;
  uint32_t flags = 0;                        // FGV_CC_*
  std::map<std::string, std::string> colls;  // name -> EP bytes ("" = the chaincode EP)
};
struct CCInfo {  // compiled
  uint8_t status = 0;  // 0 ok, 1 INVALID_CHAINCODE, 2 outside the model
  int ep = 0;
  bool colls_known = false;
  std::map<std::string, int> colls;  // -1 = the chaincode EP
  bool has_vp = false;               // the state holds key-level validation parameters of this namespace
};

struct Channel {
  std::string name;
  std::vector<Ident> idents;
  std::unordered_multimap<uint64_t, uint32_t> ident_index;
  std::unordered_map<std::string, uint32_t> canon_ids;
  std::unordered_map<std::string, int32_t> msp_ids;  // Mspid interning
  std::unordered_set<int32_t> known_msps;            // MSPs of the channel (config, declared, identities)
  RawConfig config;
  std::unordered_set<std::string> declared_msps;     // fgv_msp_declare
  std::map<std::string, CCDef> ccdefs;
  std::deque<std::string> committed_store;           // ledger txids (stable storage)
  std::unordered_set<std::string_view> committed;
  // compiled (compile())
  std::vector<Policy> policies;                      // [0] = reject
  std::unordered_map<std::string, CCInfo> ccs;
  std::unordered_map<std::string, int> implicit_ep;  // mspid -> EP of _implicit_org_<mspid>
  std::map<std::string, int> chan_idx;               // channel policy path -> index
  // committed key-level validation parameters (fgv_kvmeta_set): kvkey(ns, coll, key) -> the
  // VALIDATION_PARAMETER bytes (a SignaturePolicyEnvelope); entries per namespace
  std::unordered_map<std::string, std::string> kvmeta;
  std::unordered_map<std::string, uint32_t> kvmeta_ns;
  // compiled: kvkey -> policy index, or -3 when it does not unmarshal (the translation fails:
  // VSCCExecutionFailureError, the reference halts)
  std::unordered_map<std::string, int> kvmeta_pi;
  bool dirty = true;
  // (certifiers identifier, OU identifier) -> id, shared by identities and OU principals
  std::unordered_map<std::string, int32_t> ou_ids;
  // IDENTITY principals of channel MSPs never deserialized (compile()): the MSP cache miss
  // resolves them with a batch's identities (fgv_block_misses)
  std::vector<std::string> unresolved_principals;

  int32_t ou_intern(std::string_view certifier, std::string_view ou) {
    std::string k;
    const uint32_t a = (uint32_t)certifier.size();
    k.append(reinterpret_cast<const char *>(&a), 4).append(certifier).append(ou);
    auto it = ou_ids.find(k);
    if (it == ou_ids.end()) it = ou_ids.emplace(std::move(k), (int32_t)ou_ids.size()).first;
    return it->second;
  }

  static std::string kvkey(std::string_view ns, std::string_view coll, std::string_view key) {
    std::string k;
    k.reserve(8 + ns.size() + coll.size() + key.size());
    const uint32_t a = (uint32_t)ns.size(), b = (uint32_t)coll.size();
    k.append(reinterpret_cast<const char *>(&a), 4).append(ns).append(reinterpret_cast<const char *>(&b), 4);
    return k.append(coll).append(key);
  }
  // -1: no parameter, -3: untranslatable, else the compiled policy
  int kv_policy(std::string_view ns, std::string_view coll, std::string_view key) const {
    if (kvmeta_pi.empty()) return -1;
    auto it = kvmeta_pi.find(kvkey(ns, coll, key));
    return it == kvmeta_pi.end() ? -1 : it->second;
  }

  int32_t intern(const std::string &msp) {
    auto it = msp_ids.find(msp);
    if (it == msp_ids.end()) it = msp_ids.emplace(msp, (int32_t)msp_ids.size()).first;
    return it->second;
  }
  bool msp_known(const Span &mspid) const {
    auto it = msp_ids.find(mspid.str());
    return it != msp_ids.end() && known_msps.count(it->second) != 0;
  }
  bool is_committed(const Span &txid) const {
    return committed.count(std::string_view(reinterpret_cast<const char *>(txid.p), txid.n)) != 0;
  }
  // DeserializeIdentity over the registry: index, -1 (deserialization error: unknown MSP,
  // undecodable, or an undeserializable key), -2 (a certificate of a channel MSP that was never
  // registered: outside the engine)
  int lookup(const Span &ser) const {
    VSerializedIdentity sid;
    if (!pbw::decode(ser.p, ser.n, sid)) return -1;
    uint64_t h = hash_bytes(sid.mspid.p, sid.mspid.n);
    h = hash_bytes(sid.id_bytes.p, sid.id_bytes.n, h ^ 0xA5);
    auto range = ident_index.equal_range(h);
    for (auto it = range.first; it != range.second; ++it) {
      const Ident &I = idents[it->second];
      if (sid.mspid.eq(I.mspid.data(), I.mspid.size()) && sid.id_bytes.eq(I.id_bytes.data(), I.id_bytes.size()))
        return I.kind == FGV_KEY_UNDESERIALIZABLE ? -1 : (int)it->second;
    }
    return msp_known(sid.mspid) ? -2 : -1;
  }
  void compile();
  // compile an ApplicationPolicy into the table, returns its index
  int compile_app(const std::string &bytes);
};

constexpr const char *kImplicitPrefix = "_implicit_org_";  // core/chaincode/implicitcollection/name.go:24-29

}  // namespace fgvb
