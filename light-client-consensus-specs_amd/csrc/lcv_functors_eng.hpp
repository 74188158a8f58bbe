// lcv_functors_eng.hpp — team functors of the generated pairing programs (lcv_engine.hpp); kept
// apart from lcv_functors.hpp so that only the engine unit and the driver depend on the programs.
#pragma once
#include "lcv_engine.hpp"
#include "lcv_functors.hpp"

// pairing programs on the team engine (lcv_engine.hpp); one team of TEAM lanes per update
struct F_eng_miller {
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_MILLER_TEAM, LDS_WORDS = LCV_PROG_MILLER_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_MILLER_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_miller_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_fexp {
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_FEXP_TEAM, LDS_WORDS = LCV_PROG_FEXP_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_FEXP_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_fexp_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_h2c {
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_H2C_TEAM, LDS_WORDS = LCV_PROG_H2C_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_H2C_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_h2c_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_g2sub {
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_G2SUB_TEAM, LDS_WORDS = LCV_PROG_G2SUB_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_G2SUB_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_g2sub_team(i, lane, r, lds, cl, P, W); }
};
